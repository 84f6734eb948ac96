"""Structured metrics.

The reference's only metric is a printed job wall time (worker.py:219,234) and a
verbose-gated ``print`` logger. Here every component owns a ``Metrics`` object: thread-safe
counters, gauges and latency samples, snapshot-able as a dict and appendable as JSON lines
(``VCX_METRICS_DIR`` or an explicit path) so the coordinator and peers can be aggregated.
"""
from __future__ import annotations

import json
import os
import threading
import time

from .. import config


class Metrics:
    def __init__(self, component: str, path: str | None = None):
        self.component = component
        self._lock = threading.Lock()
        self.counters: dict[str, float] = {}
        self.gauges: dict[str, float] = {}
        self.samples: dict[str, list] = {}
        d = config.get().metrics_dir
        self.path = path or (os.path.join(d, f"{component}.jsonl") if d else None)

    def incr(self, name: str, by: float = 1):
        with self._lock:
            self.counters[name] = self.counters.get(name, 0) + by

    def gauge(self, name: str, value: float):
        with self._lock:
            self.gauges[name] = value

    def observe(self, name: str, value: float, keep: int = 10000):
        with self._lock:
            s = self.samples.setdefault(name, [])
            s.append(value)
            if len(s) > keep:
                del s[: len(s) - keep]

    def timer(self, name: str):
        m = self

        class _T:
            def __enter__(self):
                self.t0 = time.perf_counter()
                return self

            def __exit__(self, *exc):
                m.observe(name, (time.perf_counter() - self.t0) * 1e3)

        return _T()

    def snapshot(self) -> dict:
        with self._lock:
            out = {"component": self.component, "t": time.time(), "counters": dict(self.counters),
                   "gauges": dict(self.gauges)}
            for k, v in self.samples.items():
                if v:
                    sv = sorted(v)
                    out.setdefault("latency_ms", {})[k] = {
                        "n": len(sv), "mean": sum(sv) / len(sv), "p50": sv[len(sv) // 2],
                        "p99": sv[min(len(sv) - 1, int(len(sv) * 0.99))], "max": sv[-1]}
        return out

    def emit(self, **extra):
        rec = self.snapshot()
        rec.update(extra)
        if self.path:
            os.makedirs(os.path.dirname(self.path) or ".", exist_ok=True)
            with open(self.path, "a") as f:
                f.write(json.dumps(rec) + "\n")
        return rec
