"""Control-plane wire protocol (UDP datagrams), compatible with the reference.

Requests are UTF-8 datagrams ``"<verb>||<ip>:<port>"`` sent to the coordinator's control port
(default 9999); replies are ``"ok||<port>"`` for ``join`` and ``"ok"`` otherwise
(/root/reference/server.py:100-156, worker.py:50-68).

Verbs: ``join`` (enter the worker pool, get a data port), ``request`` (become a requester,
leave the pool), ``stop`` (stop requesting, back to the pool), ``end`` (leave). New verbs:
``hb`` (heartbeat; renews the lease, reply ``ok``), ``status`` (reply ``ok||<json>``), ``tjoin``
(admit a training peer ``<id>[||<token>]``; reply ``ok||<store port>||<key prefix>``), ``store``
(the same reply, for joined volunteers and admitted training peers only), ``p2p`` (reply
``ok||{"plane", "vid", "store_port", "store_prefix"}``: the data plane of this coordinator and, on the
p2p plane, the volunteer's id and the pair-rendezvous store). When the coordinator hosts a
rendezvous store, the ``join`` reply is ``ok||<port>||<key prefix>`` (the reference client reads
only the port field).

Differences from the reference, by design:
* verbs are matched EXACTLY on the field before ``||`` (the reference matches substrings, so
  an address containing "end" would be treated as the end verb);
* client retries are bounded (the reference retries forever on a 10 s select);
* a repeated ``join`` from the same address is idempotent (the reference leaks a port and
  double-inserts the client, server.py:106-109).
"""
from __future__ import annotations

import select
import socket
import time

VERBS = ("join", "request", "stop", "end", "hb", "status", "store", "p2p", "tjoin")
SEP = "||"
DEFAULT_CONTROL_PORT = 9999


def encode(verb: str, addr: str) -> bytes:
    if verb not in VERBS:
        raise ValueError(f"unknown verb {verb!r}")
    return f"{verb}{SEP}{addr}".encode("utf-8")


def decode(data: bytes):
    """-> (verb, addr) or (None, None) for a malformed datagram."""
    try:
        s = data.decode("utf-8")
    except UnicodeDecodeError:
        return None, None
    parts = s.split(SEP, 1)
    if len(parts) != 2 or parts[0] not in VERBS or not parts[1]:
        return None, None
    return parts[0], parts[1]


def reply_ok(extra: str | None = None) -> bytes:
    return ("ok" if extra is None else f"ok{SEP}{extra}").encode("utf-8")


def parse_reply(data: bytes):
    """-> (ok: bool, payload or None)"""
    s = data.decode("utf-8", "replace")
    if s == "ok":
        return True, None
    if s.startswith("ok" + SEP):
        return True, s[len("ok" + SEP):]
    return False, s


def split_store_ref(payload: str):
    """`<port>||<prefix>` (a `join` / `tjoin` / `store` reply payload) -> (port, prefix)."""
    port, _, prefix = (payload or "").partition(SEP)
    return int(port), prefix


def split_addr(addr: str):
    host, _, port = addr.rpartition(":")
    return host, int(port)


def addr_matches(addr: str, src_ip: str) -> bool:
    """Does a datagram from `src_ip` plausibly come from the volunteer that claims `addr`?
    Datagrams from this machine (loopback) are trusted; otherwise the claimed host must resolve
    to the sender's IP (a volunteer cannot act — join, request, end — on another one's behalf)."""
    if src_ip.startswith("127.") or src_ip == "::1":
        return True
    try:
        host, _ = split_addr(addr)
    except ValueError:
        return False
    if host == src_ip:
        return True
    try:
        return socket.gethostbyname(host) == src_ip
    except OSError:
        return False


class ControlClient:
    """Sends verbs to the coordinator with bounded retries (reference: unbounded)."""

    def __init__(self, server_host: str, server_port: int = DEFAULT_CONTROL_PORT, *, timeout_s: float = 2.0,
                 retries: int = 30, verbose: bool = False):
        self.addr = (server_host if server_host not in ("", "localhost") else "127.0.0.1", int(server_port))
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self.timeout_s = timeout_s
        self.retries = retries
        self.verbose = verbose

    def call(self, verb: str, my_addr: str, *, retries: int | None = None):
        """Send verb and wait for an `ok` reply. Returns the reply payload (or None)."""
        msg = encode(verb, my_addr)
        n = self.retries if retries is None else retries
        last = None
        for i in range(max(1, n)):
            if self.verbose:
                print(f"sending message trial {i}...")
            self.sock.sendto(msg, self.addr)
            t_end = time.time() + self.timeout_s
            while True:
                left = t_end - time.time()
                if left <= 0:
                    break
                ready, _, _ = select.select([self.sock], [], [], left)
                if not ready:
                    break
                data, _ = self.sock.recvfrom(65535)  # status replies can be large
                ok, payload = parse_reply(data)
                if ok:
                    return payload
                last = payload
        raise TimeoutError(f"coordinator {self.addr} did not acknowledge {verb!r} (last reply: {last!r})")

    def close(self):
        self.sock.close()


MAX_CHUNK_BYTES = 2 << 30  # the data plane's frame cap (transport.cpp max_payload default)


def valid_chunk_shape(shape, max_bytes: int = MAX_CHUNK_BYTES) -> bool:
    """A p2p chunk shape announced by a volunteer: 1-4 non-negative ints, at most `max_bytes`
    uint8 elements (the receiving volunteer allocates exactly this before the transfer)."""
    if not isinstance(shape, (list, tuple)) or not 1 <= len(shape) <= 4:
        return False
    n = 1
    for d in shape:
        if not isinstance(d, int) or isinstance(d, bool) or d < 0:
            return False
        n *= d
    return n <= max_bytes
