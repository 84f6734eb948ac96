"""Stage tracer: named spans timed with HIP events on the stream that runs them.

The reference's only timing is a wall clock around the whole video job (worker.py:105,219,234).
Here any stage can be wrapped in ``tracer.span(name)``; on a GPU the span records a start and an
end event on the current stream, so its duration is DEVICE time of the work enqueued inside it
(not host launch time), without a synchronisation per span. ``flush()`` synchronises once on the
last event, converts every pending span into one JSON line ``{component, span, start_ms, ms, ...}``
(``start_ms`` relative to the first span of the flush) and appends them to the trace file.

    tr = SpanTracer("peer0", path="gpurun_out/trace/peer0.jsonl")
    with tr.span("fwd_bwd"):
        loss = model(x, y); loss.backward()
    tr.flush(step=i)

A disabled tracer (no path, VCX_TRACE_DIR unset) costs one attribute check per span. Spans must
not be opened inside hipGraph capture (events would be captured as graph nodes); the trainer
wraps the replay as one span instead.
"""
from __future__ import annotations

import contextlib
import json
import os
import time

import torch

from .. import config


class SpanTracer:
    def __init__(self, component: str, path: str | None = None, enabled: bool | None = None):
        d = config.get().trace_dir
        self.component = component
        self.path = path or (os.path.join(d, f"{component}.jsonl") if d else None)
        self.enabled = bool(self.path) if enabled is None else enabled
        self._pending = []
        self.totals: dict[str, list] = {}  # name -> [count, total_ms]

    @contextlib.contextmanager
    def span(self, name: str):
        if not self.enabled:
            yield
            return
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            try:
                yield
            finally:
                e1.record()
                self._pending.append((name, e0, e1))
        else:
            t0 = time.perf_counter()
            try:
                yield
            finally:
                self._pending.append((name, t0, time.perf_counter()))

    def flush(self, **extra) -> list[dict]:
        if not self._pending:
            return []
        recs = []
        first = self._pending[0][1]
        if isinstance(first, torch.cuda.Event):
            self._pending[-1][2].synchronize()
            for name, e0, e1 in self._pending:
                recs.append({"component": self.component, "span": name, "start_ms": round(first.elapsed_time(e0), 4),
                             "ms": round(e0.elapsed_time(e1), 4), **extra})
        else:
            for name, t0, t1 in self._pending:
                recs.append({"component": self.component, "span": name, "start_ms": round((t0 - first) * 1e3, 4),
                             "ms": round((t1 - t0) * 1e3, 4), **extra})
        self._pending.clear()
        for r in recs:
            c = self.totals.setdefault(r["span"], [0, 0.0])
            c[0] += 1
            c[1] += r["ms"]
        if self.path:
            os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
            with open(self.path, "a") as f:
                for r in recs:
                    f.write(json.dumps(r) + "\n")
        return recs

    def summary(self) -> dict:
        return {k: {"n": n, "total_ms": round(t, 3), "mean_ms": round(t / n, 4)} for k, (n, t) in self.totals.items()}


NULL_TRACER = SpanTracer("null", enabled=False)


class HostSpans:
    """Host wall-clock busy time per named stage, summed per thread-safe stage name: where a
    pipeline thread spends its time (the device spans above time GPU work; these time what the
    host threads of a volunteer do: packing, sending, waiting for the engine, writing the sink).
    Cost: two perf_counter calls and one locked dict update per span."""

    def __init__(self):
        import threading

        self._lock = threading.Lock()
        self.totals: dict[str, list] = {}  # name -> [count, total_s, max_s]

    @contextlib.contextmanager
    def span(self, name: str):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            dt = time.perf_counter() - t0
            with self._lock:
                c = self.totals.get(name)
                if c is None:
                    self.totals[name] = [1, dt, dt]
                else:
                    c[0] += 1
                    c[1] += dt
                    c[2] = max(c[2], dt)

    def snapshot(self) -> dict:
        with self._lock:
            return {k: {"n": v[0], "total_ms": round(v[1] * 1e3, 2), "mean_ms": round(v[1] / v[0] * 1e3, 3),
                        "max_ms": round(v[2] * 1e3, 2)} for k, v in sorted(self.totals.items())}

    def reset(self):
        with self._lock:
            self.totals.clear()
