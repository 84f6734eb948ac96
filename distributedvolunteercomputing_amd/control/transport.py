"""(msg, ndarray) data plane over the native framed-TCP transport.

Drop-in for the imagezmq ``ImageHub``/``ImageSender`` pair the reference uses
(/root/reference/server.py:43,46,112,119 and worker.py:64,67,164,167): ``send_image(msg, a)``
ships a JSON header ``{msg, dtype, shape, ...meta}`` plus the raw C-contiguous buffer;
``recv_image()`` returns ``(msg, ndarray)`` viewing the received bytes without a copy.
``REQ_REP=True`` makes every send wait for the receiver's ``OK`` (the reference's flow
control); ``REQ_REP=False`` streams (the reference's PUB/SUB mode).

The byte moving is C++ (``_native.Hub`` / ``_native.Sender``): one listening socket per hub
accepts any number of senders, receive queues are bounded, all blocking I/O drops the GIL.
"""
from __future__ import annotations

import json

import numpy as np

from .. import _native_loader


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
    def __init__(self, open_port="tcp://*:5555", REQ_REP: bool = True, capacity: int = 64, bind_host: str = ""):
        N = _native_loader.native()
        self.hub = N.Hub(bind_host, _port_of(open_port), capacity, REQ_REP)
        self.req_rep = REQ_REP

    @property
    def port(self) -> int:
        return self.hub.port

    def recv_frame(self, timeout: float | None = None):
        """-> (header dict, ndarray, peer) or None on timeout/close."""
        f = self.hub.recv(-1.0 if timeout is None else float(timeout))
        if f is None:
            return None
        hdr = json.loads(f.header)
        arr = np.frombuffer(f, dtype=np.dtype(hdr.get("dtype", "uint8")))
        shape = hdr.get("shape")
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
