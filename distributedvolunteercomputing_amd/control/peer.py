"""The volunteer client: worker role (batched inference on chunks) and requester role
(capture -> chunk -> submit -> reassemble in order -> write video).

Public API kept from the reference (/root/reference/worker.py):
``client(server_ip='localhost', own_ip='localhost')``, ``.become_requester(path)``,
``.stop_requesting_thread()``, ``.exit_threads()``, ``.log(msg)``, tunables ``verbose``,
``req_rep``, ``number_of_frames_in_chunk=100``, ``max_buffer=4000``, ``my_port='5554'``; the job
prints ``final frame time taken for the job = <sec>`` like the reference.

Behavioural fixes, each deliberate:
* the first frame is processed (the reference reads it only to size the writer and drops it);
* the tail chunk (< 100 frames) is sent (the reference drops it: worker.py:126);
* chunks are contiguous [n, H, W, 3] arrays (no strip-packing index misalignment);
* a chunk is inferred as ONE batch on the GPU;
* frames are pre-resized to the 400-px annotation width on the requester (the worker would
  resize them anyway, worker.py:243), cutting the uplink ~10x for 720p input;
* heartbeats keep the lease alive; a dead worker's chunks are re-dispatched by the coordinator.

Data planes: on a ``relay`` coordinator chunk bytes go through the coordinator (host TCP, as in
the reference). On a ``p2p`` coordinator (``coordinator(data_plane="p2p")``) only metadata does:
the requester keeps each chunk in its own memory (on its GPU after the batched pre-resize) and,
when the coordinator says "send chunk c to volunteer w", posts the transfer on the pair group
requester>w (control/p2p.py; RCCL between GPU volunteers, gloo otherwise) while w posts the
matching receive; the annotated chunk comes back the same way, straight from the worker's GPU.
The requester frees a chunk when its result arrives, so a chunk whose worker died is still in
hand when the coordinator re-dispatches it.
"""
from __future__ import annotations

import json
import os
import queue
import threading
import time

import numpy as np
import torch

from .. import config
from ..io.video import open_sink, open_source
from ..jobs.video import DetectorEngine, Engine, OrderedSink
from ..ops import vision as V
from ..utils.metrics import Metrics
from ..utils.trace import HostSpans
from . import protocol
from .transport import FrameHub, FrameSender

_EMPTY = np.zeros(0, dtype=np.uint8)
# first bytes of a placeholder result (a worker asked to send a result it no longer holds): the
# pair FIFO needs a buffer of the announced shape, and the requester must tell it from a real one
_PLACEHOLDER_TAG = torch.frombuffer(bytearray(b"VCX/p2p/placeholder-result/v1\0\0"), dtype=torch.uint8)


def _placeholder(shape) -> torch.Tensor:
    t = torch.zeros(tuple(shape or (0,)), dtype=torch.uint8)
    flat = t.view(-1)
    n = min(flat.numel(), _PLACEHOLDER_TAG.numel())
    flat[:n] = _PLACEHOLDER_TAG[:n]
    return t


def _is_placeholder(buf) -> bool:
    flat = buf.reshape(-1)
    n = _PLACEHOLDER_TAG.numel()
    return flat.numel() >= n and torch.equal(flat[:n].cpu(), _PLACEHOLDER_TAG)


class _Landing:
    """A resized chunk still in flight on the requester's resize stream; ``wait()`` returns it."""

    __slots__ = ("t", "ev", "host")

    def __init__(self, t, ev, host=False):
        self.t, self.ev, self.host = t, ev, host

    @property
    def shape(self):
        return tuple(self.t.shape)

    def wait(self):
        self.ev.synchronize()
        return self.t.numpy() if self.host else self.t


def _host_tensor(a: np.ndarray) -> torch.Tensor:
    """A tensor view of a host chunk; read-only arrays (memory-mapped sources) are only ever read
    by the transfers, so torch's non-writable warning does not apply."""
    import warnings

    with warnings.catch_warnings():
        warnings.simplefilter("ignore", UserWarning)
        return torch.from_numpy(a)


class _Window:
    """A chunk that stays in its source file (shared-source mode): frames [first, first + n) of a
    memory-mapped uint8 [N, H, W, 3] .npy that every volunteer can read. The requester sends this
    index window instead of the frames; a worker reads and uploads the frames itself, over its own
    host link (the requester's single link is the ingest bound)."""

    __slots__ = ("path", "first", "n", "shape")

    def __init__(self, path: str, first: int, n: int, shape):
        self.path, self.first, self.n, self.shape = path, int(first), int(n), tuple(shape)

    def meta(self) -> dict:
        return {"path": self.path, "first": self.first, "n": self.n}

    def read(self) -> np.ndarray:
        return np.load(self.path, mmap_mode="r", allow_pickle=False)[self.first:self.first + self.n]


def _shared_path(path) -> str | None:
    """`path` resolved, if it is a .npy file under this volunteer's shared_source_root (else None):
    a worker reads windows of such files only, so a requester cannot make it read anything else."""
    root = config.get().shared_source_root
    if not root or not path:
        return None
    p, r = os.path.realpath(str(path)), os.path.realpath(root)
    if not p.endswith(".npy") or os.path.commonpath([p, r]) != r or not os.path.isfile(p):
        return None
    return p


class client:  # noqa: N801 (reference class name)
    verbose = False
    req_rep = True
    number_of_frames_in_chunk = 100
    max_buffer = 4000
    my_port = "5554"
    heartbeat_s = 1.0
    report_every = 10  # heartbeats between metrics reports to the coordinator (0: never)
    preresize = True

    def log(self, message):
        if self.verbose:
            print(message, flush=True)

    def __init__(self, server_ip: str = "localhost", own_ip: str = "localhost", *,
                 control_port: int = protocol.DEFAULT_CONTROL_PORT, my_port: int | str | None = None,
                 engine: Engine | None = None, out_dir: str = ".", out_ext: str = ".y4m",
                 verbose: bool | None = None, chunk: int | None = None, p2p_backend: str | None = None):
        if verbose is not None:
            self.verbose = verbose
        if chunk is not None:
            self.number_of_frames_in_chunk = chunk
        self.server_ip = server_ip
        self.out_dir = out_dir
        # requester-side batched pre-resize runs on the GPU when there is one (CPU volunteers
        # send raw frames; the worker resizes them as the reference does, worker.py:243)
        self.resize_device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else None
        self.out_ext = out_ext
        self.metrics = Metrics("client")
        self.hspans = HostSpans()  # host busy time per stage (bench_video.py reports it)
        self.engine = engine
        self._engine_lock = threading.Lock()
        # data port first: the coordinator connects to it while handling our join
        port = int(self.my_port if my_port is None else my_port)
        self.hub = FrameHub(port, REQ_REP=self.req_rep, capacity=8)
        self.my_ip = f"{own_ip}:{self.hub.port}"
        self.ctrl = protocol.ControlClient(server_ip, control_port, verbose=self.verbose)
        self.hb_ctrl = protocol.ControlClient(server_ip, control_port, timeout_s=0.5)  # own socket: no reply theft
        # `<port>` or `<port>||<store key prefix>` (coordinators that host a rendezvous store)
        self.connect_to_port, _, self.store_prefix = (self.ctrl.call("join", self.my_ip) or "").partition("||")
        self.sender = FrameSender(f"tcp://{server_ip}:{self.connect_to_port}", REQ_REP=self.req_rep)
        self.log(f"joined {server_ip}:{control_port}; uplink port {self.connect_to_port}, data port {self.hub.port}")
        self.plane = None
        self._outgoing: dict[int, object] = {}  # p2p: chunk key -> frames held until the result is in
        self._results: dict[int, object] = {}  # p2p: chunk id -> annotated chunk until told where to send it
        self._p2p_lock = threading.Lock()
        self._keys = iter(range(1, 1 << 62))
        self._setup_plane(server_ip, p2p_backend)

        # job state (requester role)
        self.path_out_num = 0
        self.path_out = None
        self.start_time = 0.0
        self.final_sent_frame = 0
        self.sink: OrderedSink | None = None
        self.job_times: list[float] = []

        self._pins: dict = {}  # pinned staging of the requester's pre-resize (by role)
        # memory-mapped sources page-locked in place (hipHostRegister): id -> (array, base address)
        self._registered: dict = {}
        self._win_maps: dict[str, np.ndarray] = {}  # shared-source mode: this worker's mappings by path
        # guards _registered and the enqueue of copies out of a registered mapping: a new job's
        # requester thread unregisters while the previous job's send thread may still be using it
        self._reg_lock = threading.Lock()
        self._in_done = [None, None]  # per pinned input buffer: the upload that last read it
        self._in_ring = 0
        self._rs_stream = None  # the requester's resize stream (its own: not the workers' engines')
        self.send_q: queue.Queue = queue.Queue(maxsize=self.max_buffer)
        # relay plane: packed chunks wait here for the wire thread, so packing / resizing chunk k+1
        # overlaps the uplink send of chunk k (measured serial: 9.6 + 5.2 ms per 100-frame 720p chunk,
        # the requester's send thread was the whole job's bound, profiles/r4_video_job_spans.txt)
        self.wire_q: queue.Queue = queue.Queue(maxsize=2)
        self._out_ring = 0  # pinned result buffers rotate: a packed chunk may still be queued or on the wire
        self.work_q: queue.Queue = queue.Queue(maxsize=4)
        self.continue_requesting = False
        self.continue_procesing = True
        self.continue_sending = True
        self.continue_receiving = True
        self._threads = []
        for fn, nm in ((self.worker, "worker"), (self.send_image_thread, "send"), (self._wire_thread, "wire"),
                       (self.recv_image_thread, "recv"), (self._heartbeat, "hb")):
            t = threading.Thread(target=fn, name=f"vcx-client-{nm}", daemon=True)
            t.start()
            self._threads.append(t)
        self._req_thread = None

    def _setup_plane(self, server_ip, backend):
        try:
            info = json.loads(self.ctrl.call("p2p", self.my_ip, retries=3) or "{}")
        except (TimeoutError, ValueError):
            info = {}
        if info.get("plane") != "p2p":
            return
        import datetime

        import torch.distributed as dist

        from .p2p import PairPlane

        host = server_ip if server_ip not in ("", "localhost") else "127.0.0.1"
        port = int(info["store_port"])

        prefix = info.get("store_prefix") or self.store_prefix

        def store():  # every pair-rendezvous key lives under the coordinator's secret prefix
            st = dist.TCPStore(host, port, None, False, timeout=datetime.timedelta(seconds=60))
            return dist.PrefixStore(prefix, st) if prefix else st
        if backend is None:
            # RCCL needs one GPU per volunteer; volunteers sharing a device (or none) use gloo
            backend = config.get().p2p_backend or (
                "nccl" if torch.cuda.is_available() and torch.cuda.device_count() > 1 else "gloo")
        dev = self.resize_device if backend == "nccl" else torch.device("cpu")
        self.plane = PairPlane(store, int(info["vid"]), backend=backend, device=dev, metrics=self.metrics)
        self.log(f"p2p data plane: volunteer id {self.plane.vid}, {backend} pair groups on {dev}")

    # ------------------------------------------------------------------ engine
    def _get_engine(self) -> Engine:
        with self._engine_lock:
            if self.engine is None:
                self.engine = DetectorEngine()
            return self.engine

    # ------------------------------------------------------------------ requester role
    def requester(self, path):
        os.makedirs(self.out_dir, exist_ok=True)
        self.path_out = os.path.join(self.out_dir, f"video{self.path_out_num}{self.out_ext}")
        self.path_out_num += 1
        if self.sink is not None:
            self.sink.close()
        self.final_sent_frame = 0
        with self._p2p_lock:  # chunks of an earlier job that never came back are not needed any more
            self._outgoing.clear()
        src = open_source(path)
        time.sleep(0.0 if path != "live" else 0.5)  # camera warm-up in the reference: 2 s
        # shared-source mode: on the p2p plane, chunks of a memory-mapped file under the shared root
        # go out as index windows; the workers read and upload the frames themselves
        win_path = _shared_path(getattr(src, "path", None)) if self.plane is not None else None
        # the job clock starts before the source is page-locked (reference: before the first read,
        # worker.py:105-107): that setup grows with the source and is part of the job
        self.start_time = time.time()
        if win_path is None:
            self._register_source(src)
        out_path = self.path_out

        def done(sink):
            dt = sink.t_done - self.start_time
            if sink.errors:
                # the output file is incomplete: not a completed job (no job time for it)
                self.metrics.incr("jobs_failed")
                print(f"job failed: {sink.errors} output write error(s); {out_path} is incomplete", flush=True)
                return
            self.job_times.append(dt)
            self.metrics.observe("job_s", dt)
            print(f"final frame time taken for the job = {dt}", flush=True)

        sink_dev = self.resize_device if config.get().sink_gpu else None
        self.sink = OrderedSink(lambda w, h: open_sink(out_path, w, h, 30, device=sink_dev), on_done=done)
        n = 0
        C = self.number_of_frames_in_chunk
        while self.continue_requesting:
            if win_path is not None:  # an index window: no frame byte is read or moved here
                j = src.i % len(src.a)
                arr = src.read_chunk(C)  # a view of the mapping (its pages are never touched)
                if len(arr) == 0:
                    break
                self.send_q.put(("window", (n + 1, _Window(win_path, j, len(arr), arr.shape))))
                n += len(arr)
                continue
            if src.chunked:  # whole chunks straight from the source (memory-mapped file: no copy here)
                with self.hspans.span("req_read"):
                    arr = src.read_chunk(C)
                if len(arr) == 0:
                    break
                self.send_q.put(("chunk", (n + 1, arr)))
                n += len(arr)
                continue
            with self.hspans.span("req_read"):
                ok, frame = src.read()
            if not ok:
                break
            n += 1
            self.send_q.put((n, frame))
        src.release()
        self.final_sent_frame = n
        self.send_q.put(("flush", None))
        self.sink.set_final(n)
        print(f"final frame sent : {n}\n", flush=True)
        if self.continue_requesting:  # EOF (not a user `end`)
            self.stop_requesting_thread()
        self.log("requester terminated.")

    def become_requester(self, path):
        self.ctrl.call("request", self.my_ip)
        self.continue_requesting = True
        self._req_thread = threading.Thread(target=self.requester, args=(path,), name="vcx-requester", daemon=True)
        self._req_thread.start()

    def stop_requesting_thread(self):
        self.ctrl.call("stop", self.my_ip)
        self.continue_requesting = False

    def wait_job(self, timeout: float | None = None) -> float | None:
        """Block until the current job's last frame is written; returns its wall time."""
        if self._req_thread is not None:
            self._req_thread.join(timeout)
        if self.sink is None:
            return None
        if not self.sink.done.wait(timeout):
            return None
        return self.job_times[-1] if self.job_times else None

    def _register_source(self, src):
        """Page-lock a memory-mapped source where it lies (hipHostRegister, read-only), once per job:
        each chunk's upload is then one async DMA straight out of the mapping. Without it every
        100-frame 720p chunk (276 MB) was first copied into pinned memory on the requester's send
        thread: 9.6-12.5 ms per chunk, the job's bound (profiles/r4_video_job_spans.txt).
        Mappings of earlier jobs are released first (their uploads have finished: the resize stream
        is synchronised). A failed registration leaves the copy path in place."""
        self._unregister_sources()
        a = getattr(src, "a", None)
        if (self.resize_device is None or not self.preresize or not isinstance(a, np.memmap) or a.nbytes == 0
                or not config.get().register_source):
            return
        self._register_mapping(a)

    def _register_mapping(self, a):
        """hipHostRegister (read-only) of the pages under a memory-mapped array; kept until
        _unregister_sources (next job of this requester, or exit)."""
        if not isinstance(a, np.memmap) or a.nbytes == 0:
            return
        from torch._C import _cudart

        ptr = a.__array_interface__["data"][0]
        base = ptr & ~4095  # the mapping starts on a page boundary at or before the array data
        size = ((ptr + a.nbytes - base) + 4095) & ~4095
        t0 = time.perf_counter()
        err = int(_cudart.cudaHostRegister(base, size, 0x08))  # hipHostRegisterReadOnly
        if err != 0:
            self.metrics.incr("source_register_failed")
            self.log(f"hipHostRegister of the source mapping failed ({err}): chunks are copied")
            return
        with self._reg_lock:
            self._registered[id(a)] = (a, base)
        self.metrics.observe("source_register_ms", (time.perf_counter() - t0) * 1e3)

    def _unregister_sources(self):
        """Under the registration lock: no copy out of a mapping can be enqueued between the stream
        synchronisation and the unregister (a DMA from unregistered memory can fault the GPU)."""
        with self._reg_lock:
            if not self._registered:
                return
            from torch._C import _cudart

            if self._rs_stream is not None:
                self._rs_stream.synchronize()
            if self._win_maps and torch.cuda.is_available():
                torch.cuda.synchronize()  # a worker's uploads out of a registered window mapping
            for a, base in list(self._registered.values()):
                _cudart.cudaHostUnregister(base)
            self._registered.clear()
            self._win_maps.clear()

    def _registered_block(self, frames):
        """True when `frames` is a view of a page-locked source mapping (call under _reg_lock)."""
        if not self._registered or not isinstance(frames, np.ndarray):
            return False
        b = frames
        while isinstance(b.base, np.ndarray):
            b = b.base
        return any(b is a for a, _ in list(self._registered.values())) and frames.flags.c_contiguous

    def _read_window(self, win, cshape):
        """The frames of a shared-source window as a view of this worker's mapping of the file (None when
        the window is malformed, outside this volunteer's shared_source_root, or not what was announced).
        On a GPU worker the whole mapping is page-locked once (as the requester does, _register_source),
        so each chunk's upload is one DMA out of the page cache over this worker's own link."""
        try:
            path, first, n = str(win["path"]), int(win["first"]), int(win["n"])
        except (KeyError, TypeError, ValueError):
            return None
        p = _shared_path(path)
        if p is None or first < 0 or n <= 0:
            return None
        a = self._win_maps.get(p)
        if a is None:
            try:
                a = np.load(p, mmap_mode="r", allow_pickle=False)
            except (OSError, ValueError):
                return None
            if a.ndim != 4 or a.dtype != np.uint8 or a.shape[-1] != 3:
                return None
            self._win_maps[p] = a
            eng = self.engine
            if (eng is not None and getattr(eng, "device", None) is not None and torch.device(eng.device).type == "cuda"
                    and config.get().register_source):
                self._register_mapping(a)
        if first + n > len(a):
            return None
        v = a[first:first + n]
        if cshape is not None and list(v.shape) != list(cshape):
            return None
        return v

    # ------------------------------------------------------------------ send (chunk packing)
    def send_image_thread(self):
        frames, nums = [], []
        C = self.number_of_frames_in_chunk

        def flush(block=None):
            if block is None and not frames:
                return
            first = frames[0] if block is None else block[0]
            with self.hspans.span("req_pack_resize"):
                if self.preresize and self.resize_device is not None and first.shape[1] != 400:
                    chunk = self._resize_chunk(frames if block is None else block)
                else:
                    chunk = np.stack(frames) if block is None else np.ascontiguousarray(block)
            info = f"{self.my_ip}||request||{'-'.join(map(str, nums))}||{chunk.shape[1]}||{chunk.shape[2]}"
            up = config.get().uplink_pipeline
            if up == "all" or (up == "relay" and self.plane is None):
                self.wire_q.put((info, chunk))  # in order: one wire thread
            else:
                self._ship(info, chunk)
            self.metrics.incr("chunks_sent")
            frames.clear()
            nums.clear()

        while self.continue_sending:
            try:
                item = self.send_q.get(timeout=0.2)
            except queue.Empty:
                continue
            n, f = item
            if n == "flush":
                flush()
                continue
            if n == "window":  # shared-source mode: only the chunk's index window leaves this volunteer
                flush()
                first, win = f
                info = (f"{self.my_ip}||request||{'-'.join(map(str, range(first, first + win.n)))}"
                        f"||{win.shape[1]}||{win.shape[2]}")
                key = next(self._keys)
                with self._p2p_lock:
                    self._outgoing[key] = win
                ok = self.sender.send_image(info, _EMPTY, p2p=1, key=key, cshape=list(win.shape), win=win.meta())
                if not ok:
                    self.log("uplink send failed")
                self.metrics.incr("chunks_sent")
                self.metrics.incr("window_chunks_sent")
                continue
            if n == "chunk":  # a whole chunk from a chunked source: frames first..first+k-1
                flush()
                first, block = f
                nums.extend(range(first, first + len(block)))
                flush(block)
                continue
            if frames and f.shape != frames[0].shape:
                flush()  # a chunk holds frames of one size only
            frames.append(f)
            nums.append(n)
            if len(frames) >= C:
                flush()

    def _wire_thread(self):
        """Second stage of the requester's uplink, in chunk order: waits for a chunk's resize to land
        (the send thread is already copying the next chunk into the other pinned buffer), then sends
        it (relay plane) or parks it and sends its metadata (p2p plane)."""
        while self.continue_sending:
            try:
                info, chunk = self.wire_q.get(timeout=0.2)
            except queue.Empty:
                continue
            self._ship(info, chunk)

    def _ship(self, info, chunk):
        """Send one packed chunk (relay) or park it and send its metadata (p2p)."""
        if isinstance(chunk, _Landing):
            with self.hspans.span("req_wait_resize"):
                chunk = chunk.wait()
        if self.plane is not None:  # p2p: the chunk stays here; the coordinator gets its metadata
            key = next(self._keys)
            held = chunk if isinstance(chunk, torch.Tensor) else _host_tensor(chunk)
            if held.device.type == "cpu" and self._pins and any(
                    held.data_ptr() == b.data_ptr() for b in self._pins.values()):
                held = held.clone()  # a pinned ring buffer: the next chunks reuse it (the p2p
                # path of _resize_chunk lands each chunk in a buffer of its own instead)
            with self._p2p_lock:
                self._outgoing[key] = held
            ok = self.sender.send_image(info, _EMPTY, p2p=1, key=key, cshape=list(held.shape))
        else:
            with self.hspans.span("req_send"):
                ok = self.sender.send_image(info, chunk)
        if not ok:
            self.log("uplink send failed")

    def _pinned(self, name, shape):
        b = self._pins.get(name)
        n = int(np.prod(shape))
        if b is None or b.numel() < n:
            b = self._pins[name] = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        return b[:n].view(shape)

    def _resize_chunk(self, frames):
        """One batched resize kernel per chunk on this volunteer's GPU (~10x less uplink). The
        frames are gathered straight into pinned host memory, so the upload is one async DMA (a
        pageable 276 MB 720p chunk went through a staged copy); the result comes back through
        pinned memory too, or stays on the GPU for an RCCL pair plane."""
        dev = self.resize_device
        self.metrics.incr("h2d_bytes", sum(int(f.nbytes) for f in frames) if isinstance(frames, list)
                          else int(frames.nbytes))
        if self._rs_stream is None:
            self._rs_stream = torch.cuda.Stream(dev)
        x = None
        with self._reg_lock:  # the mapping stays registered until this copy is enqueued
            if self._registered_block(frames):  # page-locked mapping: DMA straight from the source
                with torch.cuda.stream(self._rs_stream):
                    x = torch.empty(frames.shape, dtype=torch.uint8, device=dev)
                    x.copy_(_host_tensor(frames), non_blocking=True)
        if x is None:
            # two pinned input buffers: this chunk's copy overlaps the previous chunk's upload + resize
            i = self._in_ring = (self._in_ring + 1) % 2
            if self._in_done[i] is not None:
                self._in_done[i].synchronize()  # the upload that last read this buffer has finished
            pin = self._pinned(f"in{i}", (len(frames),) + tuple(frames[0].shape))
            if isinstance(frames, np.ndarray):  # one block (e.g. a memory-mapped chunk): one threaded copy
                pin.copy_(_host_tensor(frames))
            else:
                for j, f in enumerate(frames):
                    pin[j].copy_(torch.from_numpy(f))
            with torch.cuda.stream(self._rs_stream):
                x = pin.to(dev, non_blocking=True)
                up = torch.cuda.Event()
                up.record(self._rs_stream)
                self._in_done[i] = up
        with torch.cuda.stream(self._rs_stream):
            small = V.resize_width(x, 400)
            if self.plane is not None and self.plane.device.type == "cuda":
                done = torch.cuda.Event()
                done.record(self._rs_stream)
                return _Landing(small, done)  # an RCCL pair plane sends it from device memory
            if self.plane is not None:
                # a host pair plane holds the chunk until its result is back: a pinned buffer of its
                # own (torch's caching host allocator recycles them), no clone in _ship
                po = torch.empty(tuple(small.shape), dtype=torch.uint8, pin_memory=True)
            else:
                # 4 result buffers: one being sent, two queued for the wire (wire_q), one being filled
                self._out_ring = (self._out_ring + 1) % 4
                po = self._pinned(f"out{self._out_ring}", tuple(small.shape))
            po.copy_(small, non_blocking=True)
            done = torch.cuda.Event()
            done.record(self._rs_stream)
        return _Landing(po, done, host=True)

    # ------------------------------------------------------------------ receive
    def recv_image_thread(self):
        while self.continue_receiving:
            r = self.hub.recv_frame(timeout=0.2)
            if r is None:
                continue
            hdr, arr, _ = r
            if hdr.get("p2p"):
                self._p2p_command(hdr)
                continue
            parts = hdr["msg"].split("||")
            requester, command = parts[0], parts[1]
            nums = [int(x) for x in parts[2].split("-")] if parts[2] else []
            if command == "request":
                self.work_q.put((hdr, arr, requester, nums))
            elif command == "processed":
                if requester != self.my_ip or self.sink is None:
                    print("frame not mine.", flush=True)
                    continue
                self._deliver(nums, arr)

    def _deliver(self, nums, frames):
        """Hand returned frames to the in-order sink; a sink failure (e.g. an unwritable output)
        is logged and counted instead of killing the receive thread."""
        try:
            with self.hspans.span("req_sink"):
                self.sink.push_many(nums, frames)
        except Exception as e:  # noqa: BLE001
            self.metrics.incr("sink_errors")
            print(f"output sink failed: {type(e).__name__}: {e}", flush=True)

    def _p2p_command(self, hdr):
        """One coordinator instruction of the p2p plane (see the module docstring)."""
        cmd, cid = hdr.get("cmd"), int(hdr.get("chunk", -1))
        plane = self.plane
        if plane is None:
            return
        if cmd in ("work", "recv_result", "send") and not protocol.valid_chunk_shape(hdr.get("cshape")):
            self.metrics.incr("bad_frames")
            return
        if cmd == "peer_dead":
            plane.peer_dead(int(hdr["vid"]))
        elif cmd == "send":  # requester: chunk `key` -> worker `dst`
            with self._p2p_lock:
                t = self._outgoing.get(int(hdr["key"]))
            if isinstance(t, _Window):  # a worker could not read the window: send its frames after all
                self.metrics.incr("window_fallback_sends")
                t = _host_tensor(np.ascontiguousarray(t.read()))
            if t is None:
                # a chunk this requester no longer holds (an earlier job's): the worker has posted
                # the matching receive, so send a placeholder to keep the pair's FIFO in step; its
                # result lands on frames the sink has already written and is dropped there
                self.metrics.incr("p2p_placeholder_sends")
                t = torch.zeros(tuple(hdr.get("cshape") or (0,)), dtype=torch.uint8)
            plane.send(int(hdr["dst"]), t, cid)
        elif cmd == "work":  # worker: receive the chunk, then infer it
            msg = hdr["msg"]
            if hdr.get("win") is not None:  # shared-source mode: read the window from the file here
                arr = self._read_window(hdr["win"], hdr.get("cshape"))
                if arr is None:  # not readable here: the requester sends the frames instead
                    self.metrics.incr("window_refused")
                    self.sender.send_image(f"{msg.split('||')[0]}||failed", _EMPTY, p2p=1, chunk=cid, nowin=1)
                    return
                parts = msg.split("||")
                nums = [int(x) for x in parts[2].split("-")] if parts[2] else []
                self.metrics.incr("window_chunks")
                self.work_q.put(({"chunk": cid, "p2p": 1, "win": 1}, arr, parts[0], nums))
                return

            def got(buf, hdr=hdr, msg=msg):
                if isinstance(buf, BaseException):
                    # the chunk never arrived: hand it back to the coordinator, which re-queues it
                    # at the front (the requester still holds its frames)
                    self.metrics.incr("p2p_recv_failed")
                    self.sender.send_image(f"{msg.split('||')[0]}||failed", _EMPTY, p2p=1, chunk=cid)
                    return
                parts = msg.split("||")
                nums = [int(x) for x in parts[2].split("-")] if parts[2] else []
                self.work_q.put(({"chunk": cid, "p2p": 1}, buf, parts[0], nums))
            plane.recv(int(hdr["src"]), hdr["cshape"], torch.uint8, cid, got)
        elif cmd == "send_result":  # worker: annotated chunk -> requester `dst`
            with self._p2p_lock:
                t = self._results.pop(cid, None)
            if t is None:
                # the requester has posted its receive: keep the pair's FIFO in step with a
                # tagged placeholder of the announced shape; the requester recognises the tag and
                # re-submits the chunk (its frames are still held under the chunk's key)
                self.metrics.incr("p2p_placeholder_results")
                t = _placeholder(hdr.get("cshape"))
            plane.send(int(hdr["dst"]), t, cid)
        elif cmd == "recv_result":  # requester: annotated chunk from worker `src`
            key, msg = hdr.get("key"), hdr["msg"]

            def done(buf, key=key, msg=msg):
                if isinstance(buf, BaseException):
                    # the annotated chunk was lost on the way back (the worker is done with it):
                    # submit the frames again as a new chunk; they are still held under `key`
                    self.metrics.incr("p2p_recv_failed")
                    self._resubmit(key, msg)
                    return
                if _is_placeholder(buf):  # the worker no longer held the result: not frames
                    self.metrics.incr("p2p_placeholder_received")
                    self._resubmit(key, msg)
                    return
                if key is not None:
                    with self._p2p_lock:
                        self._outgoing.pop(int(key), None)
                parts = msg.split("||")
                nums = [int(x) for x in parts[2].split("-")] if parts[2] else []
                if self.sink is None or parts[0] != self.my_ip:
                    return
                self.metrics.incr("chunks_returned")
                self._deliver(nums, buf.cpu().numpy())
            plane.recv(int(hdr["src"]), hdr["cshape"], torch.uint8, cid, done)
        elif cmd == "drop":  # a duplicate result of a re-dispatched chunk: nobody wants it
            with self._p2p_lock:
                self._results.pop(cid, None)

    def _resubmit(self, key, msg):
        if key is None:
            return
        with self._p2p_lock:
            t = self._outgoing.get(int(key))
        if t is None:
            return
        parts = msg.split("||")
        info = f"{self.my_ip}||request||{parts[2]}||{t.shape[1]}||{t.shape[2]}"
        self.metrics.incr("p2p_resubmitted")
        extra = {"win": t.meta()} if isinstance(t, _Window) else {}
        self.sender.send_image(info, _EMPTY, p2p=1, key=int(key), cshape=list(t.shape), **extra)

    # ------------------------------------------------------------------ worker role
    def worker(self):
        """Worker role, two chunks deep on both planes: chunk k+1 is submitted to the engine
        before chunk k's result is collected and sent. Host chunks: k+1's host copy and H2D
        overlap k's network (DetectorEngine.submit). Device-resident chunks of the RCCL pair
        plane: k+1's compute is enqueued behind its receive while k's result is posted and sent,
        so receive k+1 ∥ infer k ∥ send k-1 (DetectorEngine.submit_tensor)."""
        pending = []
        batch_max = max(1, config.get().engine_batch)
        while self.continue_procesing:
            try:
                item = self.work_q.get(timeout=0.002 if pending else 0.2)
            except queue.Empty:
                item = None
            nxt = []
            if item is not None:
                items = [item]
                while len(items) < batch_max:  # chunks already waiting run as one network batch
                    try:
                        items.append(self.work_q.get_nowait())
                    except queue.Empty:
                        break
                nxt = self._submit(self._get_engine(), items)
            if pending and (nxt or self.work_q.empty()):
                for p in pending:
                    self._finish(*p)
                pending = []
            pending = nxt or pending
        for p in pending:
            self._finish(*p)

    def _submit(self, eng, items):
        """Submit received chunks to the engine: consecutive chunks of one kind (host / device-resident) and
        frame shape as ONE batch where the engine batches (DetectorEngine.submit_many: the network's last
        tile waves and extras tail paid once, 1.00 vs 1.16 ms per 100 frames for two chunks). Returns the
        pending (job, hdr, requester, nums, t0, dev_res) entries in arrival order."""
        groups = []
        for it in items:
            hdr, arr, _req, _nums = it
            dev_res = bool(hdr.get("p2p")) and isinstance(arr, torch.Tensor) and arr.device.type != "cpu"
            if not dev_res and getattr(eng, "device", None) is not None and torch.device(eng.device).type == "cuda":
                self.metrics.incr("h2d_bytes", int(arr.nbytes))  # this volunteer's own host -> GPU link
            if groups and groups[-1][0] == dev_res and tuple(groups[-1][1][-1][1].shape[1:]) == tuple(arr.shape[1:]):
                groups[-1][1].append(it)
            else:
                groups.append((dev_res, [it]))
        out = []
        for dev_res, its in groups:
            t0 = time.perf_counter()
            with self.hspans.span("wk_submit"):
                if not dev_res and all(h.get("win") for h, _a, _r, _n in its):
                    # shared-source windows: page-locked mapping -> upload straight from it (under the
                    # registration lock, so the mapping cannot be unregistered before the copy is enqueued)
                    jobs = []
                    for _h, a, r, _n in its:
                        with self._reg_lock:
                            jobs.append(eng.submit(a, r, pinned=self._registered_block(a)))
                elif len(its) > 1 and hasattr(eng, "submit_many"):
                    pairs = [(a, r) for _h, a, r, _n in its]
                    jobs = eng.submit_tensor_many(pairs) if dev_res else eng.submit_many(pairs)
                else:
                    jobs = [eng.submit_tensor(a, r) if dev_res else eng.submit(a, r) for _h, a, r, _n in its]
            out.extend((job, hdr, req, nums, t0, dev_res) for (hdr, _a, req, nums), job in zip(its, jobs))
        return out

    def _finish(self, job, hdr, requester, nums, t0, dev_res=False):
        if dev_res:  # annotated chunk on the device: held for the pair send to the requester
            with self.hspans.span("wk_result"):
                out = job.result()
            if out.device != self.plane.device:
                out = out.to(self.plane.device)
            self.metrics.observe("chunk_infer_ms", (time.perf_counter() - t0) * 1e3)
            self.metrics.incr("frames_processed", len(nums))
            self._post_result(hdr, out, requester, nums)
            return
        with self.hspans.span("wk_result"):
            out, counts = job.result()
        self.metrics.observe("chunk_infer_ms", (time.perf_counter() - t0) * 1e3)
        self.metrics.incr("frames_processed", len(nums))
        if hdr.get("p2p"):  # host chunk from a gloo pair: held (copied out of the pinned slot)
            self._post_result(hdr, torch.from_numpy(np.array(out)), requester, nums)
            return
        info = f"{requester}||processed||{'-'.join(map(str, nums))}||{out.shape[1]}||{out.shape[2]}"
        with self.hspans.span("wk_send"):
            self.sender.send_image(info, out, chunk=hdr.get("chunk", -1))

    def _post_result(self, hdr, out, requester, nums):
        """Hold the annotated chunk until the coordinator names its destination; report it."""
        cid = int(hdr["chunk"])
        with self._p2p_lock:
            self._results[cid] = out.contiguous()
        info = f"{requester}||processed||{'-'.join(map(str, nums))}||{out.shape[1]}||{out.shape[2]}"
        self.sender.send_image(info, _EMPTY, p2p=1, chunk=cid, cshape=list(out.shape))

    # ------------------------------------------------------------------ heartbeat / leave
    def _heartbeat(self):
        n = 0
        while self.continue_receiving:
            time.sleep(self.heartbeat_s)
            try:
                self.hb_ctrl.call("hb", self.my_ip, retries=1)
            except Exception:
                pass
            n += 1
            if self.report_every and n % self.report_every == 0:
                self.report_metrics()

    def report_metrics(self):
        """Send this volunteer's metrics snapshot to the coordinator over the data uplink (a
        metadata-only frame); the coordinator aggregates them per volunteer (status verb)."""
        snap = self.metrics.snapshot()
        snap.pop("t", None)
        try:
            return self.sender.send_image(f"{self.my_ip}||metrics", _EMPTY, metrics=snap, timeout=2.0)
        except Exception:  # noqa: BLE001 — best effort
            return False

    def exit_threads(self):
        try:
            self.ctrl.call("end", self.my_ip, retries=5)
        except TimeoutError:
            pass
        self.continue_requesting = False
        self.continue_procesing = False
        self.continue_sending = False
        self.continue_receiving = False
        for t in self._threads:
            t.join(timeout=2)
        self.hub.close()
        self.sender.close()
        if self.plane is not None:
            self.plane.close()
        if self.sink is not None:
            self.sink.close()
        self._unregister_sources()


Client = client
