"""Video sources and sinks without OpenCV/ffmpeg (neither exists on this image).

Reference: ``cv2.VideoCapture(0 | path)`` + ``cv2.VideoWriter(mp4v, 30 fps)``
(/root/reference/worker.py:95-98, 110, 215, 229). Replacements:

Sources (``open_source(spec)``):
  * ``"live"``                      — a synthetic camera (moving shapes + frame counter), endless
                                      until ``stop()``; the image has no webcam.
  * ``"synthetic:<n>[:<W>x<H>]"``   — n synthetic frames (default 1280x720).
  * ``*.y4m``                       — YUV4MPEG2 (C420jpeg/C420/C444) file, e.g. ``ffmpeg -i in.mp4 out.y4m``.
  * ``*.npy``                       — uint8 array [N, H, W, 3] (BGR, like OpenCV).
  * a directory                     — sorted image files decoded with Pillow.
All frames are H x W x 3 uint8 in **BGR** order (OpenCV's convention, which the reference's
drawing colours assume).

Sinks (``open_sink(path, width, height, fps)``):
  * ``*.y4m`` (default) — YUV4MPEG2 4:4:4, losslessly round-trippable; ``*.npy``; a directory of PNGs.
"""
from __future__ import annotations

import functools
import os
import struct
from pathlib import Path

import numpy as np


# ----------------------------------------------------------------------------- colour
def _rt():
    """The C++ runtime's colour loops (csrc/runtime/colour.cpp), or None when it is not built
    (or config.colour_native is off)."""
    from .. import config

    if not config.get().colour_native:
        return None
    try:
        from .._native_loader import native

        return native()
    except RuntimeError:
        return None


def _as_block(frames) -> np.ndarray:
    """[k, h, w, 3] contiguous: the frames' own buffer when they are consecutive views of one
    contiguous array (a received chunk), else one stacked copy."""
    f0 = frames[0]
    base = f0.base if isinstance(f0.base, np.ndarray) else None
    if base is not None and base.ndim == 4 and base.flags.c_contiguous and all(f.base is base for f in frames):
        step = f0.nbytes
        o0 = f0.__array_interface__["data"][0] - base.__array_interface__["data"][0]
        if o0 % step == 0 and all(f.__array_interface__["data"][0] == f0.__array_interface__["data"][0] + i * step
                                  for i, f in enumerate(frames)) and all(f.flags.c_contiguous for f in frames):
            j = o0 // step
            return base[j:j + len(frames)]
    return np.ascontiguousarray(np.stack(frames))


def bgr_to_yuv444(frame: np.ndarray) -> np.ndarray:
    rt = _rt()
    if rt is not None and frame.dtype == np.uint8 and frame.ndim == 3 and frame.shape[2] == 3:
        h, w = frame.shape[:2]
        out = np.empty((3, h, w), np.uint8)
        rt.bgr_to_yuv444(np.ascontiguousarray(frame), out, w, h)
        return out
    return _bgr_to_yuv444_np(frame)


def _bgr_to_yuv444_np(frame: np.ndarray) -> np.ndarray:
    f = frame.astype(np.float32)
    b, g, r = f[..., 0], f[..., 1], f[..., 2]
    y = 0.299 * r + 0.587 * g + 0.114 * b
    u = (b - y) * 0.564 + 128.0
    v = (r - y) * 0.713 + 128.0
    return np.clip(np.stack([y, u, v]) + 0.5, 0, 255).astype(np.uint8)  # [3, H, W]


def yuv444_to_bgr(yuv: np.ndarray) -> np.ndarray:
    rt = _rt()
    if rt is not None and yuv.dtype == np.uint8 and yuv.ndim == 3 and yuv.shape[0] == 3:
        h, w = yuv.shape[1:]
        yuv = np.ascontiguousarray(yuv)
        out = np.empty((h, w, 3), np.uint8)
        rt.yuv_to_bgr(yuv[0], yuv[1], yuv[2], out, w, h, w)
        return out
    return _yuv444_to_bgr_np(yuv)


def _yuv444_to_bgr_np(yuv: np.ndarray) -> np.ndarray:
    y, u, v = (yuv[i].astype(np.float32) for i in range(3))
    r = y + 1.403 * (v - 128.0)
    g = y - 0.344 * (u - 128.0) - 0.714 * (v - 128.0)
    b = y + 1.773 * (u - 128.0)
    return np.clip(np.stack([b, g, r], -1) + 0.5, 0, 255).astype(np.uint8)


# ----------------------------------------------------------------------------- sources
class FrameSource:
    chunked = False  # True: read_chunk() hands out many frames at once without a per-frame copy

    def read(self):
        """Returns (ok, frame) like cv2.VideoCapture.read()."""
        raise NotImplementedError

    def read_chunk(self, n: int):
        """Up to n frames as one [k, H, W, 3] array (k = 0 at the end)."""
        frames = []
        for _ in range(n):
            ok, f = self.read()
            if not ok:
                break
            frames.append(f)
        return np.stack(frames) if frames else np.zeros((0, 0, 0, 3), np.uint8)

    def release(self):
        pass

    def __iter__(self):
        while True:
            ok, f = self.read()
            if not ok:
                return
            yield f


@functools.lru_cache(maxsize=8)
def _gradient(width: int, height: int) -> np.ndarray:
    yy, xx = np.mgrid[0:height, 0:width]
    f = np.empty((height, width, 3), np.uint8)
    f[..., 0] = (xx * 255 // max(1, width - 1)).astype(np.uint8)
    f[..., 1] = (yy * 255 // max(1, height - 1)).astype(np.uint8)
    f[..., 2] = 0
    return f


def synthetic_frame(i: int, width: int, height: int, seed: int = 0) -> np.ndarray:
    """Deterministic test frame: gradient background, two moving boxes, frame-index bar."""
    f = _gradient(width, height).copy()
    f[..., 2] = (seed * 37 + i * 3) & 255
    bw, bh = max(4, width // 8), max(6, height // 3)
    x0 = (i * 7) % max(1, width - bw)
    y0 = height // 4
    f[y0 : y0 + bh, x0 : x0 + bw] = (40, 40, 200)
    x1 = width - bw - (i * 5) % max(1, width - bw)
    f[height // 2 : height // 2 + bh // 2, x1 : x1 + bw // 2] = (200, 200, 40)
    # frame index as a 16-bit bar code along the top rows (lets tests verify ordering)
    seg = max(1, width // 16)
    for b in range(16):
        f[0 : max(2, height // 60), b * seg : (b + 1) * seg] = 255 if (i >> b) & 1 else 0
    return f


def decode_frame_index(frame: np.ndarray, width: int | None = None) -> int:
    width = width or frame.shape[1]
    seg = max(1, width // 16)
    v = 0
    for b in range(16):
        if frame[0, b * seg + seg // 2].mean() > 127:
            v |= 1 << b
    return v


class SyntheticSource(FrameSource):
    def __init__(self, n: int | None, width: int = 1280, height: int = 720, seed: int = 0):
        self.n, self.w, self.h, self.seed, self.i = n, width, height, seed, 0
        self._stop = False

    def read(self):
        if self._stop or (self.n is not None and self.i >= self.n):
            return False, None
        f = synthetic_frame(self.i, self.w, self.h, self.seed)
        self.i += 1
        return True, f

    def release(self):
        self._stop = True


class NpySource(FrameSource):
    """Frames of a uint8 [N, H, W, 3] .npy file, memory-mapped: read_chunk() returns views into
    the mapping (no copy here; the consumer's one copy goes straight into pinned memory). With
    `total` the file is played in a loop until `total` frames (a long steady-state job from a
    file that fits in RAM: spec ``<file>.npy@<total>``)."""

    chunked = True

    def __init__(self, path, total: int | None = None):
        self.path = str(path)
        self.a = np.load(path, mmap_mode="r", allow_pickle=False)
        if self.a.ndim != 4 or self.a.shape[-1] != 3 or self.a.dtype != np.uint8:
            raise ValueError(f"{path}: expected uint8 [N,H,W,3], got {self.a.dtype} {self.a.shape}")
        self.total = len(self.a) if total is None else int(total)
        self.i = 0

    def read(self):
        if self.i >= self.total:
            return False, None
        f = np.ascontiguousarray(self.a[self.i % len(self.a)])
        self.i += 1
        return True, f

    def read_chunk(self, n: int):
        j = self.i % len(self.a)
        k = min(n, len(self.a) - j, self.total - self.i)  # a view never wraps around the file's end
        v = self.a[j : j + max(k, 0)]
        self.i += len(v)
        return v


class ImageDirSource(FrameSource):
    EXT = {".png", ".jpg", ".jpeg", ".bmp", ".ppm", ".pgm"}

    def __init__(self, path):
        self.files = sorted(p for p in Path(path).iterdir() if p.suffix.lower() in self.EXT)
        self.i = 0

    def read(self):
        from PIL import Image

        if self.i >= len(self.files):
            return False, None
        im = Image.open(self.files[self.i]).convert("RGB")
        self.i += 1
        return True, np.ascontiguousarray(np.asarray(im)[..., ::-1])


class Y4MSource(FrameSource):
    def __init__(self, path):
        self.f = open(path, "rb")
        header = self.f.readline().decode("ascii").split()
        if not header or header[0] != "YUV4MPEG2":
            raise ValueError(f"{path}: not a YUV4MPEG2 file")
        self.w = self.h = 0
        self.cs = "420jpeg"
        for tok in header[1:]:
            if tok[0] == "W":
                self.w = int(tok[1:])
            elif tok[0] == "H":
                self.h = int(tok[1:])
            elif tok[0] == "C":
                self.cs = tok[1:]

    def read(self):
        line = self.f.readline()
        if not line or not line.startswith(b"FRAME"):
            return False, None
        w, h = self.w, self.h
        if self.cs.startswith("444"):
            yuv = np.frombuffer(self.f.read(3 * w * h), np.uint8).reshape(3, h, w)
        else:  # 4:2:0 — upsample chroma by 2x2 replication
            y = np.frombuffer(self.f.read(w * h), np.uint8).reshape(h, w)
            cw, ch = (w + 1) // 2, (h + 1) // 2
            u = np.frombuffer(self.f.read(cw * ch), np.uint8).reshape(ch, cw)
            v = np.frombuffer(self.f.read(cw * ch), np.uint8).reshape(ch, cw)
            rt = _rt()
            if rt is not None:  # upsampling folded into the C++ conversion loop
                out = np.empty((h, w, 3), np.uint8)
                rt.yuv_to_bgr(y, u, v, out, w, h, cw)
                return True, out
            u = u.repeat(2, 0).repeat(2, 1)[:h, :w]
            v = v.repeat(2, 0).repeat(2, 1)[:h, :w]
            yuv = np.stack([y, u, v])
        return True, yuv444_to_bgr(yuv)

    def release(self):
        self.f.close()


def open_source(spec: str) -> FrameSource:
    if spec == "live":
        return SyntheticSource(None, 640, 480)
    if spec.startswith("synthetic"):
        parts = spec.split(":")
        n = int(parts[1]) if len(parts) > 1 and parts[1] else 300
        w, h = 1280, 720
        if len(parts) > 2:
            w, h = (int(v) for v in parts[2].lower().split("x"))
        return SyntheticSource(n, w, h)
    if "@" in spec and spec.rsplit("@", 1)[0].endswith(".npy"):  # <file>.npy@<total>: looped
        f, total = spec.rsplit("@", 1)
        return NpySource(Path(f), int(total))
    p = Path(spec)
    if p.is_dir():
        return ImageDirSource(p)
    if p.suffix == ".y4m":
        return Y4MSource(p)
    if p.suffix == ".npy":
        return NpySource(p)
    raise ValueError(f"unsupported video source {spec!r} (no OpenCV/ffmpeg here: use .y4m, .npy, an image "
                     "directory, 'live' or 'synthetic:<n>:<W>x<H>')")


# ----------------------------------------------------------------------------- sinks
def _frame_writer():
    """The C++ runtime's threaded positional frame writer (csrc/runtime/colour.cpp write_frames), or None."""
    rt = _rt()
    return rt if rt is not None and hasattr(rt, "write_frames") else None


class Y4MWriter:
    """YUV4MPEG2 4:4:4 writer (cv2.VideoWriter replacement). Every write is positional (os.pwrite at the
    writer's running offset); a received chunk's frames go through ONE native call that converts and
    writes frame ranges on several threads with the GIL released. With `device` (a GPU requester) the
    chunk's records are converted there (csrc/kernels/vision.hip bgr_to_y4m: the same bytes) and come
    back through pinned memory, so the host only copies them into the file."""

    def __init__(self, path, width, height, fps=30, device=None):
        self.device = device
        self._pin = None
        self._stream = None
        self.path, self.w, self.h = str(path), int(width), int(height)
        self.f = open(self.path, "wb")
        hdr = f"YUV4MPEG2 W{self.w} H{self.h} F{int(fps)}:1 Ip A1:1 C444\n".encode()
        os.pwrite(self.f.fileno(), hdr, 0)
        self.off = len(hdr)
        self.frames = 0

    def write(self, frame: np.ndarray):
        if frame.shape[0] != self.h or frame.shape[1] != self.w:
            raise ValueError(f"frame {frame.shape} does not match writer {self.h}x{self.w}")
        fd = self.f.fileno()
        os.pwrite(fd, b"FRAME\n", self.off)
        body = bgr_to_yuv444(frame)  # the planar buffer itself (no bytes copy)
        os.pwrite(fd, memoryview(body).cast("B"), self.off + 6)
        self.off += 6 + body.nbytes
        self.frames += 1

    def write_many(self, frames):
        """Several frames in order: one native conversion + write across threads."""
        rt = _frame_writer()
        if rt is None or any(f.shape != (self.h, self.w, 3) or f.dtype != np.uint8 for f in frames):
            for f in frames:
                self.write(f)
            return
        block = _as_block(frames)
        if self.device is not None and hasattr(rt, "write_bytes"):
            self.off += rt.write_bytes(self.f.fileno(), self.off, self._gpu_records(block))
        else:
            self.off += rt.write_frames(self.f.fileno(), self.off, block, len(block), self.w, self.h, True)
        self.frames += len(frames)

    def _gpu_records(self, block: np.ndarray) -> np.ndarray:
        import torch

        from ..ops._lib import native

        if self._stream is None:  # a stream of its own: the legacy default stream would wait for the engines
            self._stream = torch.cuda.Stream(self.device)
        with torch.cuda.device(self.device), torch.cuda.stream(self._stream):
            d = torch.from_numpy(np.ascontiguousarray(block)).to(self.device, non_blocking=True)
            rec = native().bgr_to_y4m(d)
            if self._pin is None or self._pin.numel() < rec.numel():
                self._pin = torch.empty(rec.numel(), dtype=torch.uint8, pin_memory=True)
            h = self._pin[: rec.numel()]
            h.copy_(rec, non_blocking=True)
        self._stream.synchronize()
        return h.numpy()

    def release(self):
        if self.f and not self.f.closed:
            self.f.close()


class NpyWriter:
    """uint8 [N, H, W, 3] .npy written as the frames arrive (positional writes of each received chunk,
    threaded in the C++ runtime; no copy held in memory): the header is written first with room for any
    frame count and rewritten with the final count by release()."""

    HEADER = 256  # bytes (a multiple of 64, as the format wants)

    def __init__(self, path, width, height, fps=30):
        self.path, self.w, self.h = str(path), int(width), int(height)
        self.f = open(self.path, "wb")
        self.frames = 0
        os.pwrite(self.f.fileno(), self._header(0), 0)

    def _header(self, n):
        d = "{'descr': '|u1', 'fortran_order': False, 'shape': (%d, %d, %d, 3), }" % (n, self.h, self.w)
        body = d.ljust(self.HEADER - 11) + "\n"
        return b"\x93NUMPY\x01\x00" + struct.pack("<H", len(body)) + body.encode("latin1")

    def _put(self, block):
        if block.shape[1:] != (self.h, self.w, 3) or block.dtype != np.uint8:
            raise ValueError(f"frames {block.dtype} {block.shape[1:]} do not match writer {self.h}x{self.w}")
        block = np.ascontiguousarray(block)
        off = self.HEADER + self.frames * 3 * self.w * self.h
        rt = _frame_writer()
        if rt is not None:
            rt.write_frames(self.f.fileno(), off, block, len(block), self.w, self.h, False)
        else:
            os.pwrite(self.f.fileno(), memoryview(block).cast("B"), off)
        self.frames += len(block)

    def write(self, frame):
        self._put(np.asarray(frame)[None])

    def write_many(self, frames):
        """A received chunk's frames: written straight from the chunk buffer when they are its
        consecutive views (else one stacked copy)."""
        self._put(_as_block(frames))

    def release(self):
        if self.f and not self.f.closed:
            os.pwrite(self.f.fileno(), self._header(self.frames), 0)
            self.f.close()


class PngDirWriter:
    def __init__(self, path, width, height, fps=30):
        self.dir = Path(path)
        self.dir.mkdir(parents=True, exist_ok=True)
        self.frames = 0

    def write(self, frame):
        from PIL import Image

        Image.fromarray(np.ascontiguousarray(frame[..., ::-1])).save(self.dir / f"{self.frames:06d}.png")
        self.frames += 1

    def release(self):
        pass


def open_sink(path, width, height, fps=30, device=None):
    """device: a GPU on which a Y4M sink converts its frames (None: on the host)."""
    s = str(path)
    if s.endswith(".npy"):
        return NpyWriter(path, width, height, fps)
    if s.endswith(".y4m"):
        return Y4MWriter(path, width, height, fps, device=device)
    if os.path.splitext(s)[1] == "":
        return PngDirWriter(path, width, height, fps)
    return Y4MWriter(s + ".y4m", width, height, fps, device=device)
