"""(msg, ndarray) data plane over the native framed-TCP transport.

Drop-in for the imagezmq ``ImageHub``/``ImageSender`` pair the reference uses
(/root/reference/server.py:43,46,112,119 and worker.py:64,67,164,167): ``send_image(msg, a)``
ships a JSON header ``{msg, dtype, shape, ...meta}`` plus the raw C-contiguous buffer;
``recv_image()`` returns ``(msg, ndarray)`` viewing the received bytes without a copy.
``REQ_REP=True`` makes every send wait for the receiver's ``OK`` (the reference's flow
control); ``REQ_REP=False`` streams (the reference's PUB/SUB mode).

The byte moving is C++ (``_native.Hub`` / ``_native.Sender``): one listening socket per hub
accepts any number of senders, receive queues are bounded, all blocking I/O drops the GIL.

Frames come from untrusted volunteers: the native hub drops a connection whose frame announces
more than ``max_payload`` / ``max_header`` bytes before allocating anything, and
``recv_frame`` raises ``BadFrame`` for a header that is not a JSON object, names a dtype outside
the plain numeric ones, or has a shape that does not match the payload size.
"""
from __future__ import annotations

import json

import numpy as np

from .. import _native_loader


class BadFrame(ValueError):
    """A received frame whose header is malformed or disagrees with its payload."""


# plain numeric dtypes only: no object / void / string dtypes from the wire
# (looked up by name or by the dtype's .str form; the wire string never reaches numpy's dtype
# parser, which accepts comma/repeat mini-languages and raises more than TypeError)
_DTYPE_TYPES = (np.uint8, np.int8, np.uint16, np.int16, np.uint32, np.int32, np.uint64, np.int64, np.float16,
                np.float32, np.float64, np.bool_)
_DTYPES = {np.dtype(t).str for t in _DTYPE_TYPES}
_DTYPE_BY_NAME = {k: np.dtype(t) for t in _DTYPE_TYPES for k in (np.dtype(t).name, np.dtype(t).str)}
_MAX_DIMS = 8


def decode_frame(header: str, nbytes: int):
    """-> (header dict, dtype, shape or None), validated against the payload size."""
    try:
        hdr = json.loads(header)
    except (ValueError, UnicodeDecodeError) as e:
        raise BadFrame(f"header is not JSON: {e}") from None
    if not isinstance(hdr, dict):
        raise BadFrame("header is not a JSON object")
    if not isinstance(hdr.get("msg", ""), str):
        raise BadFrame("msg must be a string")
    name = hdr.get("dtype", "uint8")
    dt = _DTYPE_BY_NAME.get(name) if isinstance(name, str) else None
    if dt is None:
        raise BadFrame(f"dtype {name!r} not allowed")
    shape = hdr.get("shape")
    if shape is not None:
        if (not isinstance(shape, list) or len(shape) > _MAX_DIMS
                or not all(isinstance(d, int) and not isinstance(d, bool) and d >= 0 for d in shape)):
            raise BadFrame(f"bad shape {shape!r}")
        if int(np.prod(shape, dtype=np.int64)) * dt.itemsize != nbytes:
            raise BadFrame(f"shape {shape} x {dt.itemsize} B != payload {nbytes} B")
    elif nbytes % dt.itemsize:
        raise BadFrame(f"payload {nbytes} B is not a multiple of {dt.itemsize}")
    return hdr, dt, shape


def _port_of(spec) -> int:
    if isinstance(spec, int):
        return spec
    s = str(spec)
    return int(s.rsplit(":", 1)[1]) if ":" in s else int(s)


def _host_of(spec) -> str:
    s = str(spec)
    if s.startswith("tcp://"):
        s = s[6:]
    return s.rsplit(":", 1)[0]


class FrameHub:
    def __init__(self, open_port="tcp://*:5555", REQ_REP: bool = True, capacity: int = 64, bind_host: str = "",
                 max_payload: int = 2 << 30, max_header: int = 64 << 10):
        N = _native_loader.native()
        self.hub = N.Hub(bind_host, _port_of(open_port), capacity, REQ_REP, int(max_payload), int(max_header))
        self.req_rep = REQ_REP

    @property
    def port(self) -> int:
        return self.hub.port

    def recv_frame(self, timeout: float | None = None):
        """-> (header dict, ndarray, peer) or None on timeout/close."""
        f = self.hub.recv(-1.0 if timeout is None else float(timeout))
        if f is None:
            return None
        view = memoryview(f)
        hdr, dt, shape = decode_frame(f.header, view.nbytes)
        arr = np.frombuffer(f, dtype=dt)
        if shape is not None:
            arr = arr.reshape(shape)
        return hdr, arr, f.peer

    def recv_image(self, timeout: float | None = None):
        r = self.recv_frame(timeout)
        if r is None:
            return None, None
        hdr, arr, _ = r
        return hdr.get("msg", ""), arr

    def send_reply(self, reply_message=b"OK"):
        """Compatibility no-op: the native hub acks each frame itself once it is queued."""

    def pending(self) -> int:
        return self.hub.pending()

    @property
    def frames_rejected(self) -> int:
        return self.hub.frames_rejected

    def close(self):
        self.hub.close()


class FrameSender:
    def __init__(self, connect_to="tcp://127.0.0.1:5555", REQ_REP: bool = True, connect_timeout: float = 10.0):
        N = _native_loader.native()
        self.sender = N.Sender(_host_of(connect_to), _port_of(connect_to), REQ_REP, connect_timeout)
        self.req_rep = REQ_REP

    def send_image(self, msg: str, image: np.ndarray, timeout: float = 120.0, **meta) -> bool:
        a = np.ascontiguousarray(image)
        hdr = {"msg": msg, "dtype": a.dtype.str, "shape": list(a.shape)}
        hdr.update(meta)
        return self.sender.send(json.dumps(hdr), a.reshape(-1).view(np.uint8) if a.size else b"", timeout)

    @property
    def connected(self) -> bool:
        return self.sender.connected

    def close(self):
        self.sender.close()
