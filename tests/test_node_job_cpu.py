"""The one-node video job (control/node_job.py): coordinator on the p2p data plane in rank 0,
every other rank a worker volunteer; chunks travel over gloo pair groups between the ranks."""
import numpy as np

from tests import _mp


def _rank(rank, world, port, out_dir, ctrl_port):
    import os

    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1")
    from distributedvolunteercomputing_amd.control.node_job import run_node_job
    from distributedvolunteercomputing_amd.jobs.video import PassthroughEngine

    return run_node_job("synthetic:230:64x48", out_dir, engine_factory=PassthroughEngine, chunk=50,
                        control_port=ctrl_port, store_port=port, lease_s=5.0, out_ext=".npy", preresize=False)


def test_node_job_over_p2p_plane(tmp_path):
    from distributedvolunteercomputing_amd.io.video import decode_frame_index

    res = _mp.run(_rank, 3, str(tmp_path), _mp.free_port(), timeout=180)
    st = res[0]
    assert st["frames"] == 230 and st["chunks"] == 5
    assert res[1] + res[2] == 230 and min(res[1], res[2]) >= 50  # both workers served chunks
    assert st["coordinator"].get("chunks_done") == 5
    frames = np.load(st["out"])
    assert [decode_frame_index(f) for f in frames] == list(range(230))
