#!/usr/bin/env python3
"""Run an N-rank RCCL job on ONE GPU (functional rehearsal of the multi-GPU paths).

RCCL refuses two ranks on one device ("Duplicate GPU detected", profiles/r2_rccl_same_gpu_probe.log):
its duplicate check compares (host hash, PCI bus id). Giving every rank its own ``NCCL_HOSTID``
makes the ranks look like separate hosts, so RCCL builds the communicator over its socket
transport on loopback instead of xGMI. That is slow, but it executes the exact c10d/RCCL code the
8-GPU driver run takes: ProcessGroupNCCL init with device_id, alltoall_base/allreduce/all-gather,
per-generation communicators, ncclCommAbort on a dead peer.

Usage: python scripts/rccl_rehearsal_launch.py --nproc 2 [--timeout 300] -- python bench.py --gpus 2 ...
This launcher never touches the GPU itself (it only spawns children), and every child gets the
torchrun-style env (RANK, LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT). Exit status: that of the
rank whose failure ended the job (128 + signal if it was killed), 124 on timeout (all children
are killed).
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--nproc", type=int, default=2)
    ap.add_argument("--timeout", type=float, default=300.0)
    ap.add_argument("--log-dir", default=None, help="per-rank stdout/stderr files (default: inherit)")
    ap.add_argument("--expect-killed", default="", help="comma-separated ranks that SIGKILL themselves on purpose "
                    "(fault-injection runs): their -9 exit does not end the job")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        ap.error("no command")
    port = free_port()
    victims = {int(r) for r in a.expect_killed.split(",") if r.strip()}
    procs = []
    for r in range(a.nproc):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.nproc), LOCAL_WORLD_SIZE=str(a.nproc),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NCCL_HOSTID=f"vcx-rehearsal-{r}",
                   NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
        out = err = None
        if a.log_dir:
            os.makedirs(a.log_dir, exist_ok=True)
            out = open(os.path.join(a.log_dir, f"rank{r}.out"), "w")
            err = open(os.path.join(a.log_dir, f"rank{r}.err"), "w")
        procs.append(subprocess.Popen(cmd, env=env, stdout=out, stderr=err, start_new_session=True))
    deadline = time.monotonic() + a.timeout
    codes = [None] * a.nproc
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None:
                codes[i] = p.poll()
        bad = [c for i, c in enumerate(codes) if c not in (None, 0) and not (i in victims and c == -signal.SIGKILL)]
        if bad or time.monotonic() > deadline:
            break
        time.sleep(0.1)
    timed_out = any(c is None for c in codes) and time.monotonic() > deadline
    first_bad = next((c for i, c in enumerate(codes) if c not in (None, 0)
                      and not (i in victims and c == -signal.SIGKILL)), None)  # the failure that ended the job
    for i, p in enumerate(procs):  # a failed or hung rank ends the whole job
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()
        codes[i] = p.returncode
    print(f"[rehearsal] rank exit codes: {codes}", file=sys.stderr, flush=True)
    if timed_out:
        return 124
    if first_bad is not None:
        return first_bad if first_bad > 0 else 128 - first_bad  # killed by a signal: 128 + signal number
    return 0


if __name__ == "__main__":
    sys.exit(main())
