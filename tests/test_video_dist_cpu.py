"""The video job over a peer group's point-to-point data plane (gloo on CPU)."""
import numpy as np

from tests import _mp


def _worker(rank, world, port, out_path):
    from distributedvolunteercomputing_amd.jobs.video import PassthroughEngine
    from distributedvolunteercomputing_amd.jobs.video_dist import run_requester, run_worker
    from distributedvolunteercomputing_amd.parallel.peer_group import PeerGroup

    store = _mp.make_store(rank, world, port)
    g = PeerGroup(store, rank, world, "gloo")
    if rank == 0:
        st = run_requester(g, "synthetic:230:64x48", out_path, "cpu", chunk=50, width=64)
        g.barrier()
        return st
    served = run_worker(g, PassthroughEngine(), "cpu")
    g.barrier()
    return {"served": served}


def test_video_job_over_p2p(tmp_path):
    out = str(tmp_path / "o.npy")
    res = _mp.run(_worker, 3, out, timeout=120)
    from distributedvolunteercomputing_amd.io.video import decode_frame_index

    assert res[0]["frames"] == 230 and res[0]["chunks"] == 5
    assert res[1]["served"] + res[2]["served"] == 5 and res[1]["served"] >= 2
    frames = np.load(out)
    assert [decode_frame_index(f) for f in frames] == list(range(230))
