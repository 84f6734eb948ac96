"""Property-based tests (hypothesis) of the pieces whose correctness is a set of invariants over
arbitrary event orders ("Chunking / reassembly — unit + property, randomized
chunk arrival order"; scheduler no-drop guarantee; wire decoding of untrusted input).

* ChunkScheduler, as a state machine driven through random interleavings of join / leave /
  lease expiry / submit / dispatch / completion / availability changes, checked against a
  plain-Python model: no chunk is ever lost or duplicated, a requester never gets its own
  chunk, per-worker credits hold, and every chunk completes once workers are available.
* OrderedSink / ReorderIndex: any arrival order with duplicates and late copies writes every
  frame exactly once, in order.
* Wire decoding: arbitrary bytes / JSON headers either decode to a consistent frame or raise
  BadFrame — never anything else.
"""
import json

import numpy as np
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st
from hypothesis.stateful import RuleBasedStateMachine, invariant, precondition, rule

from distributedvolunteercomputing_amd._native_loader import native
from distributedvolunteercomputing_amd.control import protocol
from distributedvolunteercomputing_amd.control.transport import BadFrame, decode_frame
from distributedvolunteercomputing_amd.jobs.video import OrderedSink

N = native()
NAMES = ["A", "B", "C", "D", "R1", "R2"]
CREDITS = 2


class SchedulerMachine(RuleBasedStateMachine):
    def __init__(self):
        super().__init__()
        self.s = N.ChunkScheduler(0, CREDITS)
        self.now = 0.0
        self.workers = {}  # name -> available
        self.owner = {}  # chunk -> requester
        self.inflight = {}  # chunk -> worker
        self.done = set()
        self.next_id = 1

    # ---------------------------------------------------------------- membership
    @rule(w=st.sampled_from(NAMES))
    def join(self, w):
        self.s.add_worker(w, self.now)
        self.workers.setdefault(w, True)

    @rule(w=st.sampled_from(NAMES))
    def leave(self, w):
        back = self.s.remove_worker(w)
        mine = sorted(c for c, x in self.inflight.items() if x == w)
        assert sorted(back) == mine  # exactly its in-flight chunks come back
        for c in mine:
            del self.inflight[c]
        self.workers.pop(w, None)

    @rule(w=st.sampled_from(NAMES), avail=st.booleans())
    def availability(self, w, avail):
        self.s.set_available(w, avail)
        if w in self.workers:
            self.workers[w] = avail

    @rule(dt=st.floats(min_value=0.0, max_value=3.0), beat=st.sets(st.sampled_from(NAMES)))
    def time_passes(self, dt, beat):
        self.now += dt
        for w in beat:
            self.s.heartbeat(w, self.now)
        for w in self.s.expire(self.now, 2.5):
            assert w in self.workers
            for c in [c for c, x in self.inflight.items() if x == w]:
                del self.inflight[c]
            del self.workers[w]

    # ---------------------------------------------------------------- work
    @rule(r=st.sampled_from(["R1", "R2"]))
    def submit(self, r):
        c = self.next_id
        self.next_id += 1
        self.s.submit(c, r)
        self.owner[c] = r

    @rule()
    def dispatch(self):
        a = self.s.next()
        if not a.valid():
            return
        c = a.chunk
        assert c in self.owner and c not in self.inflight and c not in self.done
        assert a.worker != self.owner[c], "a requester got its own chunk"
        assert a.requester == self.owner[c]
        assert self.workers.get(a.worker), "dispatched to an absent or unavailable worker"
        self.inflight[c] = a.worker

    @precondition(lambda self: self.inflight)
    @rule(data=st.data())
    def complete(self, data):
        c = data.draw(st.sampled_from(sorted(self.inflight)))
        assert self.s.complete(c)
        assert not self.s.complete(c)  # a duplicate completion is refused
        del self.inflight[c]
        self.done.add(c)

    # ---------------------------------------------------------------- invariants
    @invariant()
    def conservation(self):
        queued = len(self.owner) - len(self.done) - len(self.inflight)
        assert self.s.queued() == queued, "a chunk was lost or duplicated"
        assert self.s.inflight() == len(self.inflight)

    @invariant()
    def credits(self):
        for w in self.workers:
            assert self.s.inflight_of(w) <= CREDITS

    def teardown(self):
        # drain: with two available workers every remaining chunk completes
        for w in ("A", "B"):
            self.s.add_worker(w, self.now)
            self.s.set_available(w, True)
        for c in list(self.inflight):
            self.s.complete(c)
        steps = 0
        while self.s.queued() and steps < 10000:
            a = self.s.next()
            assert a.valid(), "queued chunks with an available non-requester worker must dispatch"
            assert self.s.complete(a.chunk)
            steps += 1
        assert self.s.queued() == 0 and self.s.inflight() == 0


TestSchedulerMachine = SchedulerMachine.TestCase
TestSchedulerMachine.settings = settings(max_examples=60, stateful_step_count=40, deadline=None,
                                         suppress_health_check=[HealthCheck.too_slow])


class _ListWriter:
    def __init__(self):
        self.frames = []

    def write(self, f):
        self.frames.append(int(f[0, 0, 0]))

    def release(self):
        pass


@settings(max_examples=80, deadline=None)
@given(n=st.integers(min_value=1, max_value=60), data=st.data())
def test_ordered_sink_any_arrival_order(n, data):
    frames = list(range(1, n + 1))
    order = data.draw(st.permutations(frames))
    dups = data.draw(st.lists(st.sampled_from(frames), max_size=20))
    arrivals = list(order)
    for d in dups:  # duplicates / late re-dispatched copies anywhere in the stream
        arrivals.insert(data.draw(st.integers(min_value=0, max_value=len(arrivals))), d)
    w = _ListWriter()
    sink = OrderedSink(lambda width, height: w)
    final_at = data.draw(st.integers(min_value=0, max_value=len(arrivals)))
    for i, k in enumerate(arrivals):
        if i == final_at:
            sink.set_final(n)
        sink.push(k, np.full((2, 2, 3), k % 256, dtype=np.uint8))
    if final_at >= len(arrivals):
        sink.set_final(n)
    assert sink.done.wait(10)  # the writes run on the sink's writer thread
    assert w.frames == [k % 256 for k in frames]
    assert sink.written == n and not sink.stash


class _ManyWriter(_ListWriter):
    def __init__(self):
        super().__init__()
        self.batches = 0

    def write_many(self, fs):
        self.batches += 1
        for f in fs:
            self.write(f)


@settings(max_examples=80, deadline=None)
@given(nchunks=st.integers(min_value=1, max_value=12), csize=st.integers(min_value=1, max_value=9), data=st.data())
def test_ordered_sink_chunks_any_arrival_order(nchunks, csize, data):
    """push_many (a received chunk at a time, frames handed to the writer in batches): any chunk order
    with whole-chunk duplicates writes every frame once, in order."""
    n = nchunks * csize
    chunks = [list(range(1 + c * csize, 1 + (c + 1) * csize)) for c in range(nchunks)]
    order = data.draw(st.permutations(range(nchunks)))
    dups = data.draw(st.lists(st.sampled_from(range(nchunks)), max_size=6))
    arrivals = list(order)
    for d in dups:
        arrivals.insert(data.draw(st.integers(min_value=0, max_value=len(arrivals))), d)
    w = _ManyWriter()
    sink = OrderedSink(lambda width, height: w)
    sink.set_final(n)
    for c in arrivals:
        block = np.stack([np.full((2, 2, 3), k % 256, dtype=np.uint8) for k in chunks[c]])
        sink.push_many(chunks[c], block)
    assert sink.done.wait(10)
    assert w.frames == [k % 256 for k in range(1, n + 1)]
    assert sink.written == n and not sink.stash
    assert w.batches <= nchunks


@settings(max_examples=200, deadline=None)
@given(header=st.one_of(st.text(max_size=200), st.dictionaries(
    st.sampled_from(["msg", "dtype", "shape", "chunk", "x"]),
    st.one_of(st.text(max_size=12), st.integers(-5, 10**12), st.lists(st.integers(-3, 10**7), max_size=5),
              st.none())).map(json.dumps)),
    nbytes=st.integers(min_value=0, max_value=1 << 20))
def test_decode_frame_total(header, nbytes):
    try:
        hdr, dt, shape = decode_frame(header, nbytes)
    except BadFrame:
        return
    assert isinstance(hdr, dict)
    if shape is not None:
        assert int(np.prod(shape)) * dt.itemsize == nbytes
    else:
        assert nbytes % dt.itemsize == 0


@settings(max_examples=200, deadline=None)
@given(data=st.binary(max_size=64), verb=st.sampled_from(protocol.VERBS), addr=st.text(min_size=1, max_size=40))
def test_protocol_decode_total_and_roundtrip(data, verb, addr):
    v, a = protocol.decode(data)
    assert (v is None) == (a is None)
    if v is not None:
        assert v in protocol.VERBS and a
    v2, a2 = protocol.decode(protocol.encode(verb, addr))
    assert (v2, a2) == (verb, addr)
