"""Video analytics job: per-chunk inference engines and the in-order sink.

Reference (/root/reference/worker.py:185-280): each volunteer runs, per frame,
  imutils.resize(width=400) -> blobFromImage(cv2.resize(f, (300,300)), 0.007843, mean 127.5)
  -> net.forward() -> count 'person' detections with confidence > 0.2, draw their boxes
  -> putText(requester) -> putText("person: k").
Here an engine processes a WHOLE chunk (up to 100 frames) as one batch: one H2D copy, one
batched preprocessing kernel, one batched MobileNet-SSD forward, one annotation kernel, one
D2H copy. ``DetectorEngine`` does that on the GPU with the HIP kernels (or on the CPU with
the reference ops); ``AnnotateOnlyEngine`` skips the network (used by plumbing tests).
"""
from __future__ import annotations

import threading
import time

import numpy as np
import torch

from .. import _native_loader
from ..ops import vision as V
from ..utils.trace import NULL_TRACER

PERSON = 15


class Engine:
    width = 400

    def process(self, frames: np.ndarray, requester: str) -> tuple[np.ndarray, list]:
        """frames [n, H, W, 3] uint8 BGR -> (annotated [n, h, 400, 3] uint8, per-frame counts)."""
        raise NotImplementedError

    def process_tensor(self, frames: torch.Tensor, requester: str) -> torch.Tensor:
        """Device-resident variant used by the RCCL data plane: the chunk arrives in this
        peer's memory and the annotated chunk leaves from it. Default: host round trip."""
        out, _ = self.process(frames.cpu().numpy(), requester)
        return torch.from_numpy(np.ascontiguousarray(out)).to(frames.device)

    def submit(self, frames, requester, pinned: bool = False):
        """Start a chunk; the returned job's ``result()`` gives ``process``'s return value.
        Engines without an asynchronous pipeline compute here. ``pinned``: the host frames lie in
        page-locked memory (a registered source mapping) and may be uploaded from where they are."""
        res = self.process(frames, requester)
        job = EngineJob(self, None, None, None, None)
        job.result = lambda: res
        return job

    def submit_tensor(self, frames: torch.Tensor, requester: str):
        """Device-resident variant of ``submit``: ``result()`` gives the annotated chunk as a
        tensor on the same device. Engines without an asynchronous pipeline compute here."""
        out = self.process_tensor(frames, requester)
        return _DoneJob(out)


class _DoneJob:
    def __init__(self, out):
        self.out = out

    def result(self):
        return self.out


class _TensorJob:
    """A device-resident chunk in flight on the engine's compute stream."""

    def __init__(self, out, event):
        self.out, self.event = out, event

    def result(self):
        self.event.synchronize()
        return self.out


class _Slot:
    """Pinned host staging for one in-flight chunk (input frames / annotated output)."""

    def __init__(self):
        self.pin_in = None
        self.pin_out = None
        self.h2d_done = None  # event: the pinned input may be refilled
        self.out_done = None  # event: the annotated chunk is in pin_out
        self.src_ref = None  # a caller's pinned chunk uploaded directly (kept alive until h2d_done)

    def buf(self, name, nbytes):
        b = getattr(self, name)
        if b is None or b.numel() < nbytes:
            b = torch.empty(max(nbytes, 1), dtype=torch.uint8, pin_memory=True)
            setattr(self, name, b)
        return b[:nbytes]


class EngineJob:
    """A chunk in flight on the GPU (``DetectorEngine.submit``); ``result()`` waits for it."""

    def __init__(self, engine, slot, out_shape, counts, out_dev, off: int = 0):
        self.engine, self.slot, self.out_shape, self.counts, self.out_dev = engine, slot, out_shape, counts, out_dev
        self.off = off  # byte offset of this chunk in the slot's pinned output (batched chunks share a slot)

    def result(self):
        self.slot.out_done.synchronize()
        n = int(np.prod(self.out_shape))
        out = self.slot.pin_out[self.off:self.off + n].numpy().reshape(self.out_shape)
        return out, self.counts.cpu().tolist()


class DetectorEngine(Engine):
    """Batched MobileNet-SSD volunteer engine on the GPU (or CPU reference ops).

    Stream-overlapped pipeline (SURVEY.md §2.7 "H2D copy ∥ preprocess ∥ forward ∥ send"):
    ``submit(chunk)`` copies the frames into one of two pinned staging slots (torch's threaded
    CPU copy), starts the H2D DMA on a copy stream, and enqueues resize -> blob -> network ->
    NMS -> annotation -> D2H into pinned output on the compute stream behind an event; it returns
    at once, so the caller's next chunk is copied and uploaded while this one computes.
    ``process`` = submit + result (no overlap)."""

    SLOTS = 3  # chunks in flight; a result's pinned output stays valid until SLOTS more submits

    def __init__(self, device=None, prototxt=None, caffemodel=None, conf_thresh: float = 0.2, width: int = 400,
                 consider: str = "person"):
        from ..models.mobilenet_ssd import CLASSES, SSDExecutor

        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.exec = SSDExecutor(prototxt, caffemodel, device=self.device)
        self.conf_thresh = conf_thresh
        self.width = width
        self.label = CLASSES.index(consider)
        self.consider = consider
        cuda = self.device.type == "cuda"
        self.stream = torch.cuda.Stream(self.device) if cuda else None
        self.copy_stream = torch.cuda.Stream(self.device) if cuda else None
        self._slots = [_Slot() for _ in range(self.SLOTS)] if cuda else []
        self._next = 0
        self._lock = threading.Lock()
        self.tracer = NULL_TRACER  # set a utils.trace.SpanTracer for per-stage device times

    @torch.no_grad()
    def submit(self, frames, requester, pinned: bool = False) -> "EngineJob":
        """Start a chunk ([n, H, W, 3] uint8 numpy or host tensor); returns an EngineJob. ``pinned``:
        contiguous numpy frames in page-locked memory (a hipHostRegister'ed source mapping of a shared-source
        worker) are uploaded straight from there instead of through the pinned staging slot."""
        if self.stream is None:
            out, counts = self._run(frames, requester)
            res = (out.cpu().numpy(), counts.cpu().tolist())
            job = EngineJob(self, None, None, None, None)
            job.result = lambda: res
            return job
        with self._lock:
            slot = self._slots[self._next]
            self._next = (self._next + 1) % len(self._slots)
            if slot.h2d_done is not None:
                slot.h2d_done.synchronize()  # this slot's previous upload finished
            if slot.out_done is not None:
                slot.out_done.synchronize()  # ... and its previous output was read back
            if pinned and isinstance(frames, np.ndarray) and frames.flags.c_contiguous:
                import warnings

                with warnings.catch_warnings():  # a read-only mapping: only ever read by the upload
                    warnings.simplefilter("ignore", UserWarning)
                    src = torch.from_numpy(frames)
                slot.src_ref = src
            elif isinstance(frames, torch.Tensor) and frames.is_contiguous() and frames.is_pinned():
                # already page-locked (a pinned pair-plane receive): uploaded from where it lies; the slot
                # holds the reference until the upload is known to be done
                src = frames
                slot.src_ref = frames
            else:
                a = frames if isinstance(frames, np.ndarray) else frames.numpy()
                a = np.ascontiguousarray(a)
                pin = slot.buf("pin_in", a.nbytes)
                pin.copy_(torch.from_numpy(a).view(-1).view(torch.uint8))  # threaded host copy
                src = pin.view(a.shape)
                slot.src_ref = None
            with torch.cuda.stream(self.copy_stream):
                x = src.to(self.device, non_blocking=True)
                slot.h2d_done = torch.cuda.Event()
                slot.h2d_done.record(self.copy_stream)
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(slot.h2d_done)
                x.record_stream(self.stream)
                out, counts = self._compute(x, requester)
                po = slot.buf("pin_out", out.numel()).view(out.shape)
                po.copy_(out, non_blocking=True)
                slot.out_done = torch.cuda.Event()
                slot.out_done.record(self.stream)
            return EngineJob(self, slot, tuple(out.shape), counts, out)

    @torch.no_grad()
    def process(self, frames, requester):
        return self.submit(frames, requester).result()

    @torch.no_grad()
    def process_tensor(self, frames, requester):
        """Device-resident chunk in, device-resident annotated chunk out (RCCL / IPC planes)."""
        with self._lock:
            if self.stream is None:
                out, _ = self._run(frames, requester)
                return out
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.stream):
                out, _ = self._compute(frames.to(self.device), requester)
            torch.cuda.current_stream(self.device).wait_stream(self.stream)
            return out

    @torch.no_grad()
    def submit_tensor(self, frames, requester):
        """Device-resident chunk in, annotated chunk out, asynchronously: the compute is enqueued on
        the engine's stream behind the producer of `frames` and the job's result() waits on an
        event, so a worker can receive chunk k+1 while chunk k computes and chunk k-1 is sent."""
        with self._lock:
            if self.stream is None:
                out, _ = self._run(frames, requester)
                return _DoneJob(out)
            x = frames.to(self.device)
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.stream):
                out, _ = self._compute(x, requester)
                ev = torch.cuda.Event()
                ev.record(self.stream)
            x.record_stream(self.stream)
            return _TensorJob(out, ev)

    @torch.no_grad()
    def submit_many(self, items):
        """Several host chunks [(frames, requester), ...] of one frame shape as ONE network batch: the
        per-layer kernels' last tile wave and the latency-bound extras tail are paid once per launch (two
        chunks: 1.00 vs 1.16 ms per 100 frames, profiles/r5_detector_layers.txt). One pinned slot, one
        upload, one readback; returns one job per chunk (its slice of the slot's output)."""
        shapes = [tuple(f.shape) for f, _ in items]
        if len(items) == 1 or self.stream is None or len({sh[1:] for sh in shapes}) != 1:
            return [self.submit(f, r) for f, r in items]
        with self._lock:
            slot = self._slots[self._next]
            self._next = (self._next + 1) % len(self._slots)
            if slot.h2d_done is not None:
                slot.h2d_done.synchronize()
            if slot.out_done is not None:
                slot.out_done.synchronize()
            arrs = [np.ascontiguousarray(f if isinstance(f, np.ndarray) else f.numpy()) for f, _ in items]
            pin = slot.buf("pin_in", sum(a.nbytes for a in arrs))
            off = 0
            for a in arrs:
                pin[off:off + a.nbytes].copy_(torch.from_numpy(a).view(-1).view(torch.uint8))
                off += a.nbytes
            slot.src_ref = None
            src = pin.view(sum(sh[0] for sh in shapes), *shapes[0][1:])
            with torch.cuda.stream(self.copy_stream):
                x = src.to(self.device, non_blocking=True)
                slot.h2d_done = torch.cuda.Event()
                slot.h2d_done.record(self.copy_stream)
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(slot.h2d_done)
                x.record_stream(self.stream)
                out, counts = self._compute_many(x, [r for _, r in items], [sh[0] for sh in shapes])
                po = slot.buf("pin_out", out.numel()).view(out.shape)
                po.copy_(out, non_blocking=True)
                slot.out_done = torch.cuda.Event()
                slot.out_done.record(self.stream)
            jobs, a = [], 0
            per = out[0].numel()
            for sh, c in zip(shapes, counts):
                jobs.append(EngineJob(self, slot, (sh[0],) + tuple(out.shape[1:]), c, out[a:a + sh[0]], off=a * per))
                a += sh[0]
            return jobs

    @torch.no_grad()
    def submit_tensor_many(self, items):
        """Device-resident variant of ``submit_many``: the chunks are concatenated on the device (one D2D
        copy) and run as one batch; one job per chunk (a view of the batched output)."""
        shapes = [tuple(f.shape) for f, _ in items]
        if len(items) == 1 or self.stream is None or len({sh[1:] for sh in shapes}) != 1:
            return [self.submit_tensor(f, r) for f, r in items]
        with self._lock:
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.stream):
                x = torch.cat([f.to(self.device) for f, _ in items])
                out, _ = self._compute_many(x, [r for _, r in items], [sh[0] for sh in shapes])
                ev = torch.cuda.Event()
                ev.record(self.stream)
            for f, _ in items:
                if f.device == self.device:
                    f.record_stream(self.stream)
            jobs, a = [], 0
            for sh in shapes:
                jobs.append(_TensorJob(out[a:a + sh[0]], ev))
                a += sh[0]
            return jobs

    def _compute_many(self, x, requesters, sizes):
        tr = self.tracer
        with tr.span("resize"):
            small = V.resize_width(x, self.width).contiguous()
        with tr.span("detect"):
            dets, cnt = self.exec.detect(small)
        counts, a = [], 0
        with tr.span("annotate"):
            for req, n in zip(requesters, sizes):
                counts.append(V.annotate(small[a:a + n], dets[a:a + n], cnt[a:a + n], req, label=self.label,
                                         cls_name=self.consider, thresh=self.conf_thresh))
                a += n
        return small, counts

    def _run(self, frames, requester):  # CPU path / reference
        x = frames if isinstance(frames, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(frames))
        return self._compute(x.to(self.device), requester)

    def _compute(self, x, requester):
        tr = self.tracer
        with tr.span("resize"):
            small = V.resize_width(x, self.width).contiguous()
        with tr.span("detect"):  # preprocess + MobileNet-SSD forward + decode/NMS
            dets, cnt = self.exec.detect(small)
        with tr.span("annotate"):
            counts = V.annotate(small, dets, cnt, requester, label=self.label, cls_name=self.consider,
                                thresh=self.conf_thresh)
        return small, counts


class AnnotateOnlyEngine(Engine):
    """No network: resize + annotate with zero detections (plumbing / transport tests)."""

    def __init__(self, width: int = 400, delay_s: float = 0.0):
        self.width = width
        self.delay_s = delay_s

    def process(self, frames, requester):
        x = torch.from_numpy(np.ascontiguousarray(frames))
        small = V.resize_width(x, self.width).contiguous()
        dets = torch.zeros(small.shape[0], 1, 7)
        cnt = torch.zeros(small.shape[0], dtype=torch.int32)
        counts = V.annotate(small, dets, cnt, requester)
        if self.delay_s:
            time.sleep(self.delay_s)
        return small.numpy(), counts.tolist()


class PassthroughEngine(Engine):
    """Returns frames unchanged (keeps the frame-index bar code readable for ordering tests)."""

    def __init__(self, delay_s: float = 0.0):
        self.delay_s = delay_s

    def process(self, frames, requester):
        if self.delay_s:
            time.sleep(self.delay_s)
        return np.ascontiguousarray(frames), [0] * len(frames)


class OrderedSink:
    """In-order writer (reference worker.py:210-239) on the C++ ReorderIndex: frames may arrive
    in any order, duplicates are ignored, and the job completes when the final frame lands.

    The writes run on a writer thread of their own, in order: the receive path only reorders and
    queues (a chunk's frames stay referenced, so their buffers stay alive), so receiving chunk k+1
    overlaps writing chunk k (the synchronous write held the requester's receive thread 8.7-12.5 ms
    per 100-frame chunk, profiles/r5_video_job.txt). The job is done -- and ``t_done`` taken -- once
    the writer has written the final frame and closed the file."""

    def __init__(self, writer_factory, first: int = 1, on_done=None, queue_depth: int = 4):
        import queue

        self.on_done = on_done
        self.index = _native_loader.native().ReorderIndex(first)
        self.stash: dict[int, np.ndarray] = {}
        self.writer_factory = writer_factory
        self.writer = None
        self.final = None
        self.written = 0  # frames handed to the writer
        self.errors = 0
        self.done = threading.Event()
        self.t_done = None
        self._lock = threading.Lock()
        self._finishing = False
        self._q: queue.Queue = queue.Queue(maxsize=queue_depth)
        self._thread = threading.Thread(target=self._write_loop, name="vcx-sink-writer", daemon=True)
        self._thread.start()

    _FINAL, _CLOSE = "final", "close"  # queue sentinels: job complete / sink closed early

    def _write_loop(self):
        while True:
            item = self._q.get()
            if isinstance(item, str):  # close the file; after the final frame the job is done
                if self.writer is not None:
                    try:
                        self.writer.release()
                    except Exception as e:  # noqa: BLE001
                        self.errors += 1
                        print(f"output sink failed: {type(e).__name__}: {e}", flush=True)
                if item == self._CLOSE:
                    return
                self.t_done = time.time()
                self.done.set()
                if self.on_done is not None:
                    self.on_done(self)
                return
            try:
                if hasattr(self.writer, "write_many"):
                    self.writer.write_many(item)
                else:
                    for f in item:
                        self.writer.write(f)
            except Exception as e:  # noqa: BLE001 (the job goes on; the error is counted and shown)
                self.errors += 1
                print(f"output sink failed: {type(e).__name__}: {e}", flush=True)

    def _queue(self, ready):
        if self.writer is None:
            self.writer = self.writer_factory(ready[0].shape[1], ready[0].shape[0])
        self._q.put(ready)
        self.written += len(ready)

    def set_final(self, n: int):
        with self._lock:
            self.final = n
            self._check_done()

    def push(self, n: int, frame: np.ndarray):
        self.push_many([n], [frame])

    def push_many(self, nums, frames):
        """A received chunk: every frame that becomes writable goes to the writer as one batch
        (``write_many``: one multi-threaded colour conversion and one write)."""
        with self._lock:
            ready = []
            for i, n in enumerate(nums):
                if n < self.index.next_expected or n in self.stash:
                    continue
                self.stash[n] = frames[i]
                ready.extend(self.stash.pop(k) for k in self.index.push(n))
            if ready:
                self._queue(ready)
            self._check_done()

    def _check_done(self):
        if self.final is not None and self.index.next_expected > self.final and not self._finishing:
            self._finishing = True
            self._q.put(self._FINAL)

    def close(self):
        """Stop the writer (a job that never completed: its frames so far are written) and close the file."""
        with self._lock:
            if not self._finishing:
                self._finishing = True
                self._q.put(self._CLOSE)
        self._thread.join(timeout=60)
