"""The whole volunteer video job on the GPU: coordinator + requester + 2 worker volunteers in
one process sharing the MI355X, DetectorEngine (HIP MobileNet-SSD) on every worker, on both
chunk data planes. Checks the in-order 400-px output and that every frame went through a
worker; on the p2p plane that no chunk byte crossed the coordinator."""
import numpy as np
import pytest
import torch

from distributedvolunteercomputing_amd.control.coordinator import coordinator
from distributedvolunteercomputing_amd.control.peer import client
from distributedvolunteercomputing_amd.jobs.video import DetectorEngine

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("plane", ["relay", "p2p", "p2p-rccl", "p2p-mixed"])
def test_video_job_detector_engine(gpu, tmp_path, plane):
    """p2p-rccl: the pair groups are asked for RCCL with device-resident chunks; all volunteers
    share this one GPU, so every pair detects it in the handshake and runs on gloo (host-staged)."""
    coord = coordinator("127.0.0.1", 0, ephemeral_ports=True, lease_s=5.0, data_plane=plane.split("-")[0])
    eng = DetectorEngine(device=gpu)
    backend = "nccl" if plane in ("p2p-rccl", "p2p-mixed") else None
    mk = lambda be: client("127.0.0.1", "127.0.0.1", control_port=coord.control_port, my_port=0,  # noqa: E731
                           engine=eng, out_dir=str(tmp_path), out_ext=".npy", chunk=50, p2p_backend=be)
    # p2p-mixed: an RCCL requester with gloo-only (CPU-plane) workers: the pairs negotiate gloo
    req = mk(backend)
    w1, w2 = (mk("gloo"), mk("gloo")) if plane == "p2p-mixed" else (mk(backend), mk(backend))
    try:
        req.become_requester("synthetic:230:640x360")
        t = req.wait_job(timeout=120)
        assert t is not None and t > 0
        out = np.load(req.path_out)
        assert out.shape == (230, 225, 400, 3)
        served = w1.metrics.counters.get("frames_processed", 0) + w2.metrics.counters.get("frames_processed", 0)
        assert served == 230 and req.metrics.counters.get("frames_processed", 0) == 0
        # the green "person: k" label of the annotation kernel is on every frame
        g = out[:, 180:225, 0:120]
        assert (((g[..., 1] == 255) & (g[..., 0] == 0) & (g[..., 2] == 0)).sum(axis=(1, 2)) > 10).all()
        if plane.startswith("p2p"):
            assert req.plane is not None and req.metrics.counters.get("chunks_returned", 0) == 5
        if plane == "p2p-rccl":
            assert req.plane.device.type == "cuda"
            assert req.metrics.counters.get("p2p_same_device_pairs", 0) >= 2
        if plane == "p2p-mixed":
            assert req.metrics.counters.get("p2p_mixed_backend_pairs", 0) >= 2
    finally:
        for c in (req, w1, w2):
            c.exit_threads()
        coord.exit_threads()


def test_y4m_sink_gpu_records_equal_host(tmp_path):
    """The Y4M sink's GPU conversion (csrc/kernels/vision.hip bgr_to_y4m) writes the same bytes as the host
    conversion (csrc/runtime/colour.cpp), odd sizes and a partial last write included."""
    import numpy as np

    from distributedvolunteercomputing_amd.io.video import Y4MWriter

    rng = np.random.default_rng(7)
    frames = rng.integers(0, 256, (23, 37, 53, 3), dtype=np.uint8)
    paths = []
    for dev in (None, torch.device("cuda", 0)):
        p = tmp_path / f"{'gpu' if dev is not None else 'host'}.y4m"
        w = Y4MWriter(p, 53, 37, device=dev)
        w.write_many(list(frames[:10]))
        w.write(frames[10])
        w.write_many(list(frames[11:]))
        w.release()
        paths.append(p)
    assert paths[0].read_bytes() == paths[1].read_bytes()


def test_engine_batch_matches_per_chunk(gpu):
    """DetectorEngine.submit_many / submit_tensor_many (a worker holding several chunks runs them as ONE network
    batch, config.engine_batch) give each chunk the frames and counts of its own per-chunk submit."""
    eng = DetectorEngine(device=gpu)
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (40, 225, 400, 3), dtype=np.uint8)
    b = rng.integers(0, 256, (24, 225, 400, 3), dtype=np.uint8)
    ra, rca = eng.submit(a, "alice").result()
    ra = ra.copy()
    rb, rcb = eng.submit(b, "bob").result()
    rb = rb.copy()
    ja, jb = eng.submit_many([(a, "alice"), (b, "bob")])
    (oa, ca), (ob, cb) = ja.result(), jb.result()
    for o, r in ((oa, ra), (ob, rb)):
        assert o.shape == r.shape
        assert (o != r).mean() < 1e-3  # split-K counts of the small layers may differ with the batch size
    assert len(ca) == 40 and len(cb) == 24
    assert sum(x != y for x, y in zip(ca + cb, rca + rcb)) <= 1
    ta, tb = torch.from_numpy(a).to(gpu), torch.from_numpy(b).to(gpu)
    jt = eng.submit_tensor_many([(ta, "alice"), (tb, "bob")])
    for j, r in zip(jt, (ra, rb)):
        t = j.result().cpu().numpy()
        assert t.shape == r.shape and (t != r).mean() < 1e-3
