"""C++ runtime (scheduler, reorder index, transport) and control protocol, on CPU."""
import threading
import time

import numpy as np
import pytest

from distributedvolunteercomputing_amd._native_loader import native
from distributedvolunteercomputing_amd.control import protocol
from distributedvolunteercomputing_amd.control.transport import FrameHub, FrameSender

N = native()


def test_round_robin_excludes_requester_and_never_drops():
    s = N.ChunkScheduler(0, 0)
    s.submit(1, "R")
    assert not s.next().valid()  # empty pool: the chunk waits (reference drops it)
    for w in ("R", "A", "B"):
        s.add_worker(w, 0.0)
    got = []
    for c in range(2, 8):
        s.submit(c, "R")
    while True:
        a = s.next()
        if not a.valid():
            break
        got.append((a.chunk, a.worker))
        assert a.worker != "R"
    assert [c for c, _ in got] == list(range(1, 8))
    ws = [w for _, w in got]
    assert ws == ["A", "B"] * 3 + ["A"]  # strict alternation at chunk granularity


def test_credits_and_completion():
    s = N.ChunkScheduler(0, 1)
    s.add_worker("A", 0.0)
    s.submit(1, "R")
    s.submit(2, "R")
    a = s.next()
    assert a.valid() and a.chunk == 1
    assert not s.next().valid()  # A is at its credit limit
    assert s.complete(1)
    assert not s.complete(1)  # duplicate completion is ignored
    assert s.next().chunk == 2


def test_worker_loss_requeues_in_order():
    s = N.ChunkScheduler(0, 4)
    s.add_worker("A", 0.0)
    s.add_worker("B", 0.0)
    for c in range(1, 5):
        s.submit(c, "R")
    assigned = [s.next() for _ in range(4)]
    a_chunks = sorted(x.chunk for x in assigned if x.worker == "A")
    back = s.remove_worker("A")
    assert sorted(back) == a_chunks
    again = [s.next() for _ in range(len(a_chunks))]
    assert [x.chunk for x in again] == a_chunks and all(x.worker == "B" for x in again)


def test_lease_expiry():
    s = N.ChunkScheduler(0, 2)
    s.add_worker("A", 0.0)
    s.add_worker("B", 0.0)
    s.heartbeat("B", 5.0)
    assert s.expire(6.0, 3.0) == ["A"]
    assert s.workers() == ["B"]


def test_least_loaded_policy():
    s = N.ChunkScheduler(1, 0)
    for w in ("A", "B", "C"):
        s.add_worker(w, 0)
    for c in range(6):
        s.submit(c, "R")
    ws = [s.next().worker for _ in range(6)]
    assert sorted(ws) == ["A", "A", "B", "B", "C", "C"]


def test_reorder_index():
    r = N.ReorderIndex(1)
    assert r.push(3) == []
    assert r.push(2) == []
    assert r.push(1) == [1, 2, 3]
    assert r.push(2) == []  # late duplicate
    assert r.push(5) == [] and r.stashed == 1
    assert r.push(4) == [4, 5]


def test_transport_roundtrip_ack_and_many_senders():
    hub = FrameHub(0, REQ_REP=True, capacity=4)
    senders = [FrameSender(f"tcp://127.0.0.1:{hub.port}") for _ in range(3)]
    arrs = [np.random.randint(0, 255, (5, 7, 3), dtype=np.uint8) for _ in range(3)]

    def send(i):
        assert senders[i].send_image(f"m{i}", arrs[i], chunk=i)

    th = [threading.Thread(target=send, args=(i,)) for i in range(3)]
    for t in th:
        t.start()
    got = {}
    for _ in range(3):
        hdr, a, peer = hub.recv_frame(timeout=5)
        got[hdr["chunk"]] = (hdr["msg"], a.copy())
    for t in th:
        t.join()
    for i in range(3):
        assert got[i][0] == f"m{i}" and np.array_equal(got[i][1], arrs[i])
    big = np.random.rand(1000, 1000).astype(np.float32)
    assert senders[0].send_image("big", big)
    msg, a = hub.recv_image(timeout=5)
    assert msg == "big" and a.dtype == np.float32 and np.array_equal(a, big)
    assert hub.recv_image(timeout=0.05) == (None, None)
    hub.close()


def test_transport_backpressure_and_timeout():
    hub = FrameHub(0, REQ_REP=True, capacity=1)
    s = FrameSender(f"tcp://127.0.0.1:{hub.port}")
    x = np.zeros(10, np.uint8)
    assert s.send_image("a", x, timeout=2)
    t0 = time.time()
    assert not s.send_image("b", x, timeout=0.5)  # queue full: no ack -> bounded wait, not a hang
    assert time.time() - t0 < 3
    hub.close()


def test_protocol_exact_verbs():
    assert protocol.decode(b"join||1.2.3.4:5554") == ("join", "1.2.3.4:5554")
    assert protocol.decode(b"joined||x") == (None, None)  # no substring matching
    assert protocol.decode(b"end") == (None, None)
    assert protocol.parse_reply(b"ok||5555") == (True, "5555")
    assert protocol.parse_reply(b"ok") == (True, None)
    with pytest.raises(ValueError):
        protocol.encode("bogus", "x")


def test_span_tracer_jsonl(tmp_path):
    """utils/trace.py: spans become JSONL records with durations; disabled tracers record nothing."""
    import json

    from distributedvolunteercomputing_amd.utils.trace import NULL_TRACER, SpanTracer

    p = tmp_path / "t" / "peer0.jsonl"
    tr = SpanTracer("peer0", path=str(p))
    for _ in range(2):
        with tr.span("a"):
            sum(range(1000))
        with tr.span("b"):
            pass
    recs = tr.flush(step=3)
    assert [r["span"] for r in recs] == ["a", "b", "a", "b"]
    assert all(r["ms"] >= 0 and r["step"] == 3 for r in recs)
    lines = [json.loads(x) for x in p.read_text().splitlines()]
    assert len(lines) == 4 and lines[0]["component"] == "peer0"
    assert tr.summary()["a"]["n"] == 2
    with NULL_TRACER.span("x"):
        pass
    assert NULL_TRACER.flush() == []


def _raw_frame(header: bytes, payload: bytes, payload_len=None, header_len=None, magic=0x56435846):
    import struct

    hl = len(header) if header_len is None else header_len
    pl = len(payload) if payload_len is None else payload_len
    return struct.pack("<IIQ", magic, hl, pl) + header + payload


def _send_raw(port, data, read_ack=False):
    import socket

    s = socket.create_connection(("127.0.0.1", port), timeout=2)
    s.sendall(data)
    s.settimeout(2)
    try:
        got = s.recv(16)  # "OK" for an accepted frame, b"" once the hub drops the connection
    except (ConnectionResetError, socket.timeout):
        got = b""
    s.close()
    return got


def test_transport_rejects_oversized_and_malformed_frames():
    """Untrusted volunteers: an announced 1 TB payload or 1 GB header is refused before any
    allocation (the connection is dropped, the hub keeps serving); malformed JSON / dtype /
    shape headers raise BadFrame instead of killing the ingest loop."""
    import resource

    from distributedvolunteercomputing_amd.control.transport import BadFrame

    hub = FrameHub(0, REQ_REP=True, capacity=4, max_payload=1 << 20)
    rss0 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
    assert _send_raw(hub.port, _raw_frame(b"{}", b"", payload_len=1 << 40)) == b""
    assert _send_raw(hub.port, _raw_frame(b"", b"", header_len=1 << 30)) == b""
    assert _send_raw(hub.port, _raw_frame(b"{}", b"", magic=0x1234)) == b""
    time.sleep(0.2)
    assert hub.frames_rejected == 3
    assert resource.getrusage(resource.RUSAGE_SELF).ru_maxrss - rss0 < 200_000  # KiB: nothing near 1 TB / 1 GB
    bad = [
        (b"not json", b"\x00" * 4),
        (b"[1, 2]", b"\x00" * 4),
        (b'{"msg": "x", "dtype": "O", "shape": [1]}', b"\x00" * 8),
        (b'{"msg": "x", "dtype": "<f4", "shape": [3]}', b"\x00" * 8),  # 12 B announced, 8 B sent
        (b'{"msg": "x", "dtype": "|u1", "shape": [-2, -4]}', b"\x00" * 8),
        (b'{"msg": 5}', b""),
    ]
    for h, p in bad:
        assert _send_raw(hub.port, _raw_frame(h, p)) == b"OK"  # framing is fine: queued
        with pytest.raises(BadFrame):
            hub.recv_frame(timeout=2)
    # the hub still works for a well-formed sender
    s = FrameSender(f"tcp://127.0.0.1:{hub.port}")
    x = np.arange(12, dtype=np.int16).reshape(3, 4)
    assert s.send_image("good", x)
    hdr, a, _ = hub.recv_frame(timeout=2)
    assert hdr["msg"] == "good" and np.array_equal(a, x)
    hub.close()


def test_coordinator_ignores_unjoined_and_bad_frames():
    import socket

    from distributedvolunteercomputing_amd.control.coordinator import coordinator

    c = coordinator("127.0.0.1", control_port=0, ephemeral_ports=True, lease_s=30)
    try:
        cs = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        cs.settimeout(2)
        for verb in ("request", "stop", "end", "hb"):
            cs.sendto(f"{verb}||10.9.9.9:5554".encode(), ("127.0.0.1", c.control_port))
            ok, payload = protocol.parse_reply(cs.recvfrom(4096)[0])
            assert not ok and "not joined" in payload
        assert c.metrics.snapshot()["counters"]["unknown_datagrams"] == 4
        assert protocol.addr_matches("10.0.0.5:5554", "10.0.0.5")
        assert not protocol.addr_matches("10.0.0.5:5554", "10.0.0.6")
        assert protocol.addr_matches("10.0.0.5:5554", "127.0.0.1")  # local sender: trusted
    finally:
        c.exit_threads()



def test_valid_chunk_shape():
    assert protocol.valid_chunk_shape([100, 225, 400, 3])
    assert protocol.valid_chunk_shape((0,))
    for bad in (None, [], [1, 2, 3, 4, 5], [-1, 3], [2.5, 3], ["3"], [True], [1 << 20, 1 << 20, 3], "abc"):
        assert not protocol.valid_chunk_shape(bad), bad
