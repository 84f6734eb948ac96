"""End-to-end volunteer video job on CPU: coordinator + volunteers over the UDP control verbs
(reference server.py/worker.py flow), on both data planes: ``relay`` (chunk
bytes through the coordinator's native TCP hubs) and ``p2p`` (metadata through the coordinator,
chunk bytes over directional gloo pair groups between the volunteers)."""
import time

import numpy as np
import pytest

from distributedvolunteercomputing_amd.control.coordinator import coordinator
from distributedvolunteercomputing_amd.control.peer import client
from distributedvolunteercomputing_amd.io.video import decode_frame_index
from distributedvolunteercomputing_amd.jobs.video import AnnotateOnlyEngine, PassthroughEngine


@pytest.fixture(params=["relay", "p2p"])
def coord(request):
    c = coordinator("127.0.0.1", 0, ephemeral_ports=True, lease_s=2.0, data_plane=request.param)
    yield c
    c.exit_threads()


def _client(coord, tmp_path, engine, chunk=100):
    c = client("127.0.0.1", "127.0.0.1", control_port=coord.control_port, my_port=0, engine=engine,
               out_dir=str(tmp_path), out_ext=".npy", chunk=chunk)
    c.heartbeat_s = 0.2
    return c


def test_join_request_and_inorder_output(coord, tmp_path):
    req = _client(coord, tmp_path, PassthroughEngine())
    w1 = _client(coord, tmp_path, PassthroughEngine(delay_s=0.05))
    w2 = _client(coord, tmp_path, PassthroughEngine())
    try:
        assert len(coord.sched.workers()) == 3
        req.preresize = False
        req.become_requester("synthetic:250:64x48")
        t = req.wait_job(timeout=60)
        assert t is not None and t > 0
        out = np.load(req.path_out)
        assert out.shape == (250, 48, 64, 3)  # tail chunk of 50 frames is NOT dropped
        idx = [decode_frame_index(f) for f in out]
        assert idx == list(range(250))  # in-order reassembly, first frame kept
        # the requester itself never received work; both workers did
        assert w1.metrics.counters.get("frames_processed", 0) + w2.metrics.counters.get("frames_processed", 0) == 250
        assert req.metrics.counters.get("frames_processed", 0) == 0
        assert coord.clients and req.my_ip in coord.clients  # back in the pool after EOF (stop verb)
        if coord.data_plane == "p2p":  # no chunk byte went through the coordinator
            assert all(c.plane is not None for c in (req, w1, w2))
            assert req.metrics.counters.get("chunks_returned", 0) == 3
            assert not req._outgoing and not w1._results and not w2._results
    finally:
        for c in (req, w1, w2):
            c.exit_threads()


def test_annotated_output_is_400_wide(coord, tmp_path):
    req = _client(coord, tmp_path, AnnotateOnlyEngine())
    w = _client(coord, tmp_path, AnnotateOnlyEngine())
    try:
        req.become_requester("synthetic:30:640x360")
        assert req.wait_job(timeout=60) is not None
        out = np.load(req.path_out)
        assert out.shape == (30, 225, 400, 3)
        # green "person: 0" label pixels exist near the bottom-left
        g = out[0, 180:225, 0:120]
        assert ((g[..., 1] == 255) & (g[..., 0] == 0) & (g[..., 2] == 0)).sum() > 10
    finally:
        req.exit_threads()
        w.exit_threads()


def test_dead_worker_chunks_are_redispatched(coord, tmp_path):
    req = _client(coord, tmp_path, PassthroughEngine())
    good = _client(coord, tmp_path, PassthroughEngine(delay_s=0.02))
    bad = _client(coord, tmp_path, PassthroughEngine())
    try:
        # "crash" the bad worker: it swallows work and stops heartbeating, never says `end`
        bad.continue_procesing = False
        bad.continue_receiving = False
        time.sleep(0.3)
        req.preresize = False
        req.become_requester("synthetic:400:32x24")
        t = req.wait_job(timeout=90)
        assert t is not None, "job must complete despite a dead worker"
        out = np.load(req.path_out)
        assert [decode_frame_index(f) for f in out] == list(range(400))
        assert coord.metrics.counters.get("leaves_lease", 0) >= 1
    finally:
        for c in (req, good, bad):
            c.exit_threads()


def test_two_requesters_at_once(coord, tmp_path):
    """Two volunteers submit videos concurrently (reference: several requesters interleave in
    one FIFO, server.py:24,56,80-82); each gets its own frames back, in order, every frame
    processed exactly once."""
    a = _client(coord, tmp_path / "a", PassthroughEngine(), chunk=30)
    b = _client(coord, tmp_path / "b", PassthroughEngine(), chunk=30)
    w = _client(coord, tmp_path / "w", PassthroughEngine(delay_s=0.01), chunk=30)
    try:
        for c in (a, b):
            c.preresize = False
        a.become_requester("synthetic:150:32x24")
        b.become_requester("synthetic:95:48x32")
        assert a.wait_job(timeout=60) is not None and b.wait_job(timeout=60) is not None
        oa, ob = np.load(a.path_out), np.load(b.path_out)
        assert oa.shape == (150, 24, 32, 3) and ob.shape == (95, 32, 48, 3)
        assert [decode_frame_index(f) for f in oa] == list(range(150))
        assert [decode_frame_index(f) for f in ob] == list(range(95))
        # a requester whose video is done is back in the pool (stop verb) and may serve the other
        assert sum(c.metrics.counters.get("frames_processed", 0) for c in (a, b, w)) == 245
    finally:
        for c in (a, b, w):
            c.exit_threads()


def test_volunteer_metrics_aggregated_at_coordinator(coord, tmp_path):
    req = _client(coord, tmp_path, PassthroughEngine())
    w = _client(coord, tmp_path, PassthroughEngine())
    try:
        req.preresize = False
        req.become_requester("synthetic:120:32x24")
        assert req.wait_job(timeout=60) is not None
        assert w.report_metrics() and req.report_metrics()
        t0 = time.time()
        while time.time() - t0 < 10:
            rep = coord.status()["peers"]
            if len(rep["volunteers"]) == 2 and rep["totals"].get("frames_processed") == 120:
                break
            time.sleep(0.05)
        rep = coord.status()["peers"]
        assert rep["volunteers"][w.my_ip]["counters"]["frames_processed"] == 120
        assert rep["totals"]["chunks_sent"] == 2 and rep["totals"]["frames_processed"] == 120
        # the status VERB (one UDP datagram) carries the per-volunteer reports too
        import json

        from distributedvolunteercomputing_amd.control import protocol

        st = json.loads(protocol.ControlClient("127.0.0.1", coord.control_port).call("status", "x:0"))
        assert st["peers"]["totals"]["frames_processed"] == 120 and len(st["peers"]["volunteers"]) == 2
    finally:
        for c in (req, w):
            c.exit_threads()
    assert coord.status()["peers"]["volunteers"] == {}  # gone with the volunteers


def test_status_and_idempotent_join(coord, tmp_path):
    w = _client(coord, tmp_path, PassthroughEngine())
    try:
        from distributedvolunteercomputing_amd.control import protocol

        cc = protocol.ControlClient("127.0.0.1", coord.control_port)
        p1 = cc.call("join", w.my_ip)
        p2 = cc.call("join", w.my_ip)
        assert p1 == p2 and p1.split("||")[0] == w.connect_to_port  # port [|| store key prefix]
        assert coord.sched.workers().count(w.my_ip) == 1
        import json

        st = json.loads(cc.call("status", w.my_ip))
        assert w.my_ip in st["workers"]
    finally:
        w.exit_threads()


def _worker_proc(port, delay, q):
    import os
    import time as _t

    os.environ.setdefault("OMP_NUM_THREADS", "1")
    from distributedvolunteercomputing_amd.control.peer import client as _client_cls
    from distributedvolunteercomputing_amd.jobs.video import PassthroughEngine as _PE

    c = _client_cls("127.0.0.1", "127.0.0.1", control_port=port, my_port=0, engine=_PE(delay_s=delay))
    c.heartbeat_s = 0.2
    q.put(c.my_ip)
    while True:
        _t.sleep(1)


def test_p2p_worker_process_killed_mid_transfer(tmp_path):
    """p2p plane, real crash: a worker PROCESS is SIGKILLed while it holds chunks; its pair
    groups die with it, the coordinator's lease expiry re-dispatches its chunks, and the
    requester (which still holds them) sends them to the surviving worker."""
    import multiprocessing as mp
    import os
    import signal

    c = coordinator("127.0.0.1", 0, ephemeral_ports=True, lease_s=1.5, data_plane="p2p")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker_proc, args=(c.control_port, d, q), daemon=True) for d in (0.05, 0.3)]
    for p in procs:
        p.start()
    req = None
    try:
        addrs = [q.get(timeout=120) for _ in procs]
        req = _client(c, tmp_path, PassthroughEngine())
        req.preresize = False
        req.become_requester("synthetic:600:32x24")
        slow = None
        t0 = time.time()
        while time.time() - t0 < 30 and slow is None:  # kill whichever worker holds chunks first... the slow one
            for a in addrs:
                if c.sched.inflight_of(a) > 0 and a == addrs[1]:
                    slow = a
            time.sleep(0.01)
        assert slow is not None
        os.kill(procs[1].pid, signal.SIGKILL)
        t = req.wait_job(timeout=90)
        assert t is not None, "job must complete after a worker process was killed"
        out = np.load(req.path_out)
        assert [decode_frame_index(f) for f in out] == list(range(600))
        cnt = c.metrics.counters
        assert cnt.get("leaves_lease", 0) + cnt.get("leaves_broken", 0) >= 1, sorted(cnt.items())  # expired or send failed
        assert cnt.get("redispatched", 0) >= 1, cnt
        assert req.metrics.counters.get("p2p_failed", 0) >= 1 or cnt.get("duplicate_results", 0) == 0
    finally:
        if req is not None:
            req.exit_threads()
        for p in procs:
            if p.is_alive():
                p.kill()
            p.join(timeout=5)
        c.exit_threads()


def test_streaming_transport_mode(tmp_path):
    """The reference's PUB/SUB alternative (``req_rep = False``): frames stream without per-frame
    acks; the job still completes in order."""
    class C(coordinator):
        req_rep = False

    class V(client):
        req_rep = False

    c = C("127.0.0.1", 0, ephemeral_ports=True, lease_s=2.0)
    mk = lambda e: V("127.0.0.1", "127.0.0.1", control_port=c.control_port, my_port=0, engine=e,  # noqa: E731
                     out_dir=str(tmp_path), out_ext=".npy", chunk=40)
    req, w = mk(PassthroughEngine()), mk(PassthroughEngine())
    try:
        req.preresize = False
        req.become_requester("synthetic:130:32x24")
        assert req.wait_job(timeout=60) is not None
        out = np.load(req.path_out)
        assert [decode_frame_index(f) for f in out] == list(range(130))
    finally:
        req.exit_threads()
        w.exit_threads()
        c.exit_threads()


def test_p2p_transfer_failure_between_live_volunteers_is_redispatched(tmp_path):
    """on the p2p plane a transfer that fails between two LIVE volunteers must not lose
    its chunk. The worker's first receive fails like a broken transport; it reports the chunk back
    (`failed`), the coordinator re-queues it at the front, both ends rebuild the pair under a new
    generation, and the job completes with every frame in order."""
    c = coordinator("127.0.0.1", 0, ephemeral_ports=True, lease_s=5.0, data_plane="p2p")
    req = _client(c, tmp_path, PassthroughEngine(), chunk=30)
    w = _client(c, tmp_path, PassthroughEngine(), chunk=30)
    try:
        assert w.plane is not None
        w.plane.inject_failures = 1
        req.preresize = False
        req.become_requester("synthetic:90:32x24")
        assert req.wait_job(timeout=90) is not None, "job must complete despite the failed transfer"
        out = np.load(req.path_out)
        assert [decode_frame_index(f) for f in out] == list(range(90))
        assert w.metrics.counters.get("p2p_recv_failed", 0) == 1
        assert c.metrics.counters.get("p2p_failed_requeued", 0) == 1
        assert w.plane.inject_failures == 0
    finally:
        req.exit_threads()
        w.exit_threads()
        c.exit_threads()


def test_memory_mapped_npy_source_sends_whole_chunks(coord, tmp_path):
    """A .npy video is read as memory-mapped chunks (one copy per chunk, no per-frame copy); the
    tail chunk, the frame numbering and the in-order output are unchanged."""
    from distributedvolunteercomputing_amd.io.video import synthetic_frame

    src = tmp_path / "in.npy"
    np.save(src, np.stack([synthetic_frame(i, 64, 48) for i in range(230)]))
    req = _client(coord, tmp_path, PassthroughEngine())
    w = _client(coord, tmp_path, PassthroughEngine())
    try:
        req.preresize = False
        req.become_requester(str(src))
        assert req.wait_job(timeout=60) is not None
        out = np.load(req.path_out)
        assert out.shape == (230, 48, 64, 3)
        assert [decode_frame_index(f) for f in out] == list(range(230))
        assert req.metrics.counters.get("chunks_sent", 0) == 3
    finally:
        req.exit_threads()
        w.exit_threads()


def test_failed_output_writes_fail_the_job(coord, tmp_path, monkeypatch):
    """a sink whose writes fail (disk full, I/O error) must not record a completed job
    time for a truncated output file."""
    import distributedvolunteercomputing_amd.control.peer as peer_mod

    class Broken:
        def write(self, f):
            raise OSError(28, "No space left on device")

        def release(self):
            pass

    monkeypatch.setattr(peer_mod, "open_sink", lambda *a, **k: Broken())
    req = _client(coord, tmp_path, PassthroughEngine())
    w = _client(coord, tmp_path, PassthroughEngine())
    try:
        req.preresize = False
        req.become_requester("synthetic:120:64x48")
        assert req.wait_job(timeout=60) is None  # done, but not a completed job
        assert req.sink.done.is_set() and req.sink.errors > 0
        assert req.job_times == [] and req.metrics.counters.get("jobs_failed", 0) == 1
    finally:
        for c in (req, w):
            c.exit_threads()


def _p2p_coord():
    return coordinator("127.0.0.1", 0, ephemeral_ports=True, lease_s=2.0, data_plane="p2p")


def test_shared_source_windows_leave_the_requester_without_frames(tmp_path):
    """with the source under the shared root, the requester sends only index windows;
    each worker reads its chunks' frames from the file itself. Three volunteers; the requester reads and
    moves no frame byte, the output is complete and in order. Reference: every chunk went through the
    requester and the coordinator (/root/reference/worker.py:131-159, server.py:84-90)."""
    from distributedvolunteercomputing_amd import config
    from distributedvolunteercomputing_amd.io.video import synthetic_frame

    src = tmp_path / "shared" / "in.npy"
    src.parent.mkdir()
    np.save(src, np.stack([synthetic_frame(i, 64, 48) for i in range(230)]))
    c = _p2p_coord()
    req = _client(c, tmp_path, PassthroughEngine())
    w1 = _client(c, tmp_path, PassthroughEngine())
    w2 = _client(c, tmp_path, PassthroughEngine(delay_s=0.02))
    try:
        with config.override(shared_source_root=str(src.parent)):
            req.preresize = False
            req.become_requester(str(src))
            assert req.wait_job(timeout=60) is not None
        out = np.load(req.path_out)
        assert [decode_frame_index(f) for f in out] == list(range(230))
        rc = req.metrics.counters
        assert rc.get("window_chunks_sent", 0) == 3 and rc.get("chunks_returned", 0) == 3
        assert rc.get("h2d_bytes", 0) == 0 and rc.get("window_fallback_sends", 0) == 0
        assert c.metrics.counters.get("window_dispatched", 0) == 3
        assert sum(w.metrics.counters.get("window_chunks", 0) for w in (w1, w2)) == 3
        assert sum(w.metrics.counters.get("frames_processed", 0) for w in (w1, w2)) == 230
        assert not req._outgoing  # every window released once its result was in
    finally:
        for v in (req, w1, w2):
            v.exit_threads()
        c.exit_threads()


def test_worker_that_cannot_read_the_window_gets_the_frames_from_the_requester(tmp_path):
    """A worker outside the shared root (or without the file) refuses the window; the coordinator turns
    that chunk into an ordinary pair transfer and the requester reads and sends its frames."""
    from distributedvolunteercomputing_amd import config
    from distributedvolunteercomputing_amd.io.video import synthetic_frame

    src = tmp_path / "shared" / "in.npy"
    src.parent.mkdir()
    np.save(src, np.stack([synthetic_frame(i, 32, 24) for i in range(200)]))
    c = _p2p_coord()
    req = _client(c, tmp_path, PassthroughEngine(), chunk=40)
    w = _client(c, tmp_path, PassthroughEngine(), chunk=40)
    w._read_window = lambda *a, **k: None  # this worker cannot see the file
    try:
        with config.override(shared_source_root=str(src.parent)):
            req.preresize = False
            req.become_requester(str(src))
            assert req.wait_job(timeout=60) is not None
        out = np.load(req.path_out)
        assert [decode_frame_index(f) for f in out] == list(range(200))
        assert w.metrics.counters.get("window_refused", 0) == 5
        assert req.metrics.counters.get("window_fallback_sends", 0) == 5
        assert c.metrics.counters.get("window_fallbacks", 0) == 5
    finally:
        req.exit_threads()
        w.exit_threads()
        c.exit_threads()


def test_window_outside_the_shared_root_is_refused(tmp_path):
    from distributedvolunteercomputing_amd import config
    from distributedvolunteercomputing_amd.control.peer import _shared_path

    inside = tmp_path / "root" / "a.npy"
    inside.parent.mkdir()
    np.save(inside, np.zeros((2, 4, 4, 3), np.uint8))
    outside = tmp_path / "b.npy"
    np.save(outside, np.zeros((2, 4, 4, 3), np.uint8))
    with config.override(shared_source_root=str(inside.parent)):
        assert _shared_path(str(inside)) == str(inside.resolve())
        assert _shared_path(str(outside)) is None
        assert _shared_path(str(inside.parent / ".." / "b.npy")) is None  # no escape through ..
    with config.override(shared_source_root=""):
        assert _shared_path(str(inside)) is None  # off unless a root is configured
