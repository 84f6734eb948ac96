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


class DetectorEngine(Engine):
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
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        self._lock = threading.Lock()
        self.tracer = NULL_TRACER  # set a utils.trace.SpanTracer for per-stage device times

    @torch.no_grad()
    def process(self, frames, requester):
        with self._lock:
            if self.stream is not None:
                with torch.cuda.stream(self.stream):
                    out, counts = self._run(frames, requester)
                self.stream.synchronize()
            else:
                out, counts = self._run(frames, requester)
            return out.cpu().numpy(), counts.cpu().tolist()

    @torch.no_grad()
    def process_tensor(self, frames, requester):
        with self._lock:
            out, _ = self._run(frames, requester)
            return out

    def _staging(self, nbytes):
        """Reusable pinned host buffer: one DMA-able copy per chunk instead of pin_memory()."""
        buf = getattr(self, "_pinned", None)
        if buf is None or buf.numel() < nbytes:
            buf = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
            self._pinned = buf
        return buf[:nbytes]

    def _run(self, frames, requester):
        tr = self.tracer
        with tr.span("h2d"):
            if isinstance(frames, torch.Tensor):
                x = frames.to(self.device)
            else:
                a = np.ascontiguousarray(frames)
                if self.device.type == "cuda":
                    st = self._staging(a.nbytes)
                    torch.cuda.current_stream().synchronize()  # previous chunk's H2D done before reuse
                    st.numpy()[:] = a.reshape(-1)
                    x = st.view(a.shape).to(self.device, non_blocking=True)
                else:
                    x = torch.from_numpy(a)
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
    in any order, duplicates are ignored, and the job completes when the final frame lands."""

    def __init__(self, writer_factory, first: int = 1, on_done=None):
        self.on_done = on_done
        self.index = _native_loader.native().ReorderIndex(first)
        self.stash: dict[int, np.ndarray] = {}
        self.writer_factory = writer_factory
        self.writer = None
        self.final = None
        self.written = 0
        self.done = threading.Event()
        self.t_done = None
        self._lock = threading.Lock()

    def set_final(self, n: int):
        with self._lock:
            self.final = n
            self._check_done()

    def push(self, n: int, frame: np.ndarray):
        with self._lock:
            if n < self.index.next_expected or n in self.stash:
                return
            self.stash[n] = frame
            for k in self.index.push(n):
                f = self.stash.pop(k)
                if self.writer is None:
                    self.writer = self.writer_factory(f.shape[1], f.shape[0])
                self.writer.write(f)
                self.written += 1
            self._check_done()

    def _check_done(self):
        if self.final is not None and self.index.next_expected > self.final and not self.done.is_set():
            self.t_done = time.time()
            if self.writer is not None:
                self.writer.release()
            self.done.set()
            if self.on_done is not None:
                self.on_done(self)

    def close(self):
        with self._lock:
            if self.writer is not None:
                self.writer.release()
