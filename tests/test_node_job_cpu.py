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


def test_video_cli_three_processes_exit_cleanly(tmp_path):
    """The `video` command as three separate processes (torchrun-style env, gloo pairs): every
    volunteer exits 0 (a gloo pair group left to interpreter finalisation used to abort the
    process with "terminate called without an active exception")."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, os.path.join(root, "scripts", "rccl_rehearsal_launch.py"), "--nproc", "3", "--timeout",
           "150", "--log-dir", str(tmp_path), "--", sys.executable, "-u", "-m",
           "distributedvolunteercomputing_amd.cli.main", "video", "--source", "synthetic:80:96x64", "--out-dir",
           str(tmp_path), "--out-ext", ".npy", "--chunk", "40", "--port", str(_mp.free_port()), "--store-port",
           str(_mp.free_port())]
    env = dict(os.environ, VCX_P2P_BACKEND="gloo")
    r = subprocess.run(cmd, cwd=root, capture_output=True, text=True, timeout=200, env=env)
    errs = "".join((tmp_path / f"rank{i}.err").read_text()[-1500:] for i in range(3))
    assert r.returncode == 0, r.stderr + errs
    assert "terminate called" not in errs


def _rank_npy(rank, world, port, out_dir, ctrl_port, src):
    import os

    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1")
    from distributedvolunteercomputing_amd.control.node_job import run_node_job
    from distributedvolunteercomputing_amd.jobs.video import PassthroughEngine

    st = run_node_job(src, out_dir, engine_factory=PassthroughEngine, chunk=50, control_port=ctrl_port,
                      store_port=port, lease_s=5.0, out_ext=".npy", preresize=False)
    return st


def test_node_job_npy_source_is_read_by_the_workers(tmp_path):
    """VERDICT r5 next #4 (8-GPU-shaped ingest): with an .npy source, node_job puts every volunteer in
    shared-source mode; the requester (rank 0) sends index windows only, each worker reads its chunks
    from the file, and the output is complete and in order."""
    from distributedvolunteercomputing_amd.io.video import decode_frame_index, synthetic_frame

    src = tmp_path / "src" / "in.npy"
    src.parent.mkdir()
    np.save(src, np.stack([synthetic_frame(i, 64, 48) for i in range(230)]))
    out = tmp_path / "out"
    out.mkdir()
    res = _mp.run(_rank_npy, 3, str(out), _mp.free_port(), str(src), timeout=180)
    st = res[0]
    assert st["frames"] == 230 and st["chunks"] == 5
    assert st["requester"].get("window_chunks_sent") == 5 and st["requester"].get("h2d_bytes", 0) == 0
    assert st["coordinator"].get("window_dispatched") == 5 and not st["coordinator"].get("window_fallbacks")
    frames = np.load(st["out"])
    assert [decode_frame_index(f) for f in frames] == list(range(230))
