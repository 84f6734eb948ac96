#!/usr/bin/env python3
"""Headline benchmark: GPT-2-small local-SGD training throughput (samples/s) on N MI355X peers.

BASELINE.json metric: "samples/sec GPT-2-small local-SGD at 1/2/4/8 peers; step-time under
1-peer drop". Config 2: GPT-2-small bf16, one volunteer peer per GPU, local-SGD with H=4 local
AdamW steps between averaging rounds over RCCL/xGMI.

One "step" = one local AdamW step of every peer (fwd + bwd + fused AdamW on the full model);
every H-th step additionally runs the averaging round, which is therefore inside the timed
region at its real 1/H frequency. Weak scaling: per-peer batch is fixed, global batch = N x B.

Contract (driver): `python bench.py --gpus N --steps K --warmup W`, one rank per GPU. Under
torchrun (WORLD_SIZE set) this process is one rank. Without a launcher and N > 1, this process
touches no GPU: it starts `torch.distributed.run` with N ranks as a CHILD process (never an exec)
and exits with its status, so `--gpus N` always means N ranks. A rank whose formed process group
is not N ranks exits non-zero. Rank 0 prints ONE JSON line; `value` is the whole-job samples/s,
`rccl_world` the size of the process group that actually formed, `devices` each rank's device.
Reference analog: round-robin over every available volunteer, /root/reference/server.py:84-90.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time


def _visible_gpus() -> int:
    """GPUs this process could use, counted without the HIP runtime (the spawning parent must make
    no HIP call at all): the *_VISIBLE_DEVICES lists when set, else the KFD
    topology in sysfs (GPU nodes have SIMDs). 0 = none found / unknown: the ranks validate."""
    lists = [os.environ[v] for v in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")
             if v in os.environ]
    if lists:
        return min(len([x for x in v.split(",") if x.strip()]) for v in lists)
    n = 0
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        for node in os.listdir(base):
            try:
                with open(os.path.join(base, node, "properties")) as f:
                    props = dict(ln.split()[:2] for ln in f if len(ln.split()) >= 2)
            except OSError:
                continue
            if int(props.get("simd_count", "0")) > 0:
                n += 1
    except OSError:
        return 0
    return n


def _mapped_libs() -> list[str]:
    try:
        with open("/proc/self/maps") as f:
            return sorted({ln.split()[-1].rsplit("/", 1)[-1] for ln in f if ".so" in ln})
    except OSError:
        return []


def _spawn_ranks(n: int, argv) -> int:
    """Launch n ranks of this script through torch.distributed.run in a child process. The parent
    imports neither torch nor the HIP runtime (it counts GPUs from the environment / sysfs)."""
    ndev = _visible_gpus()
    if 0 < ndev < n:
        print(f"[bench] --gpus {n} but only {ndev} GPUs are visible", file=sys.stderr)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver (RCCL)
    rc = subprocess.call(cmd, env=env)
    rep = os.environ.get("VCX_BENCH_PARENT_LIBS")
    if rep:  # tests/test_bench_cpu.py: what the spawning parent had mapped
        with open(rep, "w") as f:
            f.write("\n".join(_mapped_libs()) + "\n")
    return rc


if __name__ == "__main__" and "WORLD_SIZE" not in os.environ:
    _pre = argparse.ArgumentParser(add_help=False)
    _pre.add_argument("--gpus", type=int, default=1)
    _n = _pre.parse_known_args()[0].gpus
    if _n > 1:
        sys.exit(_spawn_ranks(_n, sys.argv[1:]))

from distributedvolunteercomputing_amd.utils.tuning import enable_tuned_gemms  # noqa: E402

TUNED_GEMMS = enable_tuned_gemms(int(os.environ.get("LOCAL_RANK", "0")))  # before torch's first GEMM

import torch  # noqa: E402
import torch.distributed as dist

from distributedvolunteercomputing_amd.models.gpt2 import GPT2, GPT2Config
from distributedvolunteercomputing_amd.ops.linear import gemm_choices
from distributedvolunteercomputing_amd.parallel.local_sgd import LocalSGDConfig, LocalSGDTrainer
from distributedvolunteercomputing_amd.parallel.peer_group import PeerGroup

BF16_DENSE_PEAK = 2.5e15  # MI355X dense bf16 MFMA, no sparsity


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--model", default="gpt2")
    ap.add_argument("--batch", type=int, default=64, help="per-peer micro-batch (sequences)")
    ap.add_argument("--seq", type=int, default=1024)
    ap.add_argument("--H", type=int, default=4)
    ap.add_argument("--algo", default="direct", choices=["rccl", "rs_ag", "butterfly", "ring", "direct"],
                    help="averaging all-reduce: direct = one-shot all-to-all reduce-scatter/all-gather over "
                         "all 7 xGMI links (parallel/collectives.py); rccl = the library all-reduce")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--graph", type=int, default=1, help="1: replay each local step as one hipGraph, 0: eager")
    ap.add_argument("--rccl-log", type=int, default=1,
                    help="1: RCCL INIT/P2P log to a file per rank (unless NCCL_DEBUG is set), parsed for the "
                         "transport each connection chose (rccl_transports in the JSON)")
    return ap.parse_args()


def _rccl_log_setup(enable: bool, rank: int) -> str | None:
    if not enable or "NCCL_DEBUG" in os.environ:
        return None
    d = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"vcx_bench_rccl_{os.getppid()}")
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, f"rank{rank}.log")
    os.environ.update(NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT,P2P,NET", NCCL_DEBUG_FILE=path)
    return path


def _rccl_transports(path: str | None) -> dict:
    """Counts of the transports RCCL's connection lines name ('... via P2P/IPC', 'via SHM', 'via NET/...')."""
    import re

    out: dict[str, int] = {}
    if not path or not os.path.exists(path):
        return out
    with open(path, errors="replace") as f:
        for ln in f:
            m = re.search(r" via (\S+)", ln)
            if m and "Channel" in ln:
                out[m.group(1)] = out.get(m.group(1), 0) + 1
    try:
        os.remove(path)
    except OSError:
        pass
    return out


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus != world:
        print(f"[bench] --gpus {a.gpus} but the launch formed WORLD_SIZE={world}", file=sys.stderr)
        return 3
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    rccl_log = _rccl_log_setup(a.rccl_log and world > 1, rank)
    cuda = torch.cuda.is_available()
    if cuda:
        # one rank per GPU; ranks beyond the GPU count share cards (rehearsal launches only)
        device = torch.device("cuda", local % torch.cuda.device_count())
        torch.cuda.set_device(device)
    else:
        device = torch.device("cpu")
    if world > 1:
        dist.init_process_group("nccl" if cuda else "gloo", device_id=device if cuda else None)
        formed = dist.get_world_size()
        if formed != a.gpus:
            print(f"[bench] process group formed {formed} ranks, --gpus {a.gpus}", file=sys.stderr)
            return 3
        if cuda:
            # one GPU per rank whenever there are enough GPUs: two ranks on one card would halve
            # that card's share and report a per-GPU number that is not one
            ndev = torch.cuda.device_count()
            p = torch.cuda.get_device_properties(device)
            mine = (device.index, getattr(p, "pci_bus_id", None), getattr(p, "uuid", None))
            seen = [None] * formed
            dist.all_gather_object(seen, str(mine))
            if formed <= ndev and len(set(seen)) < formed:
                print(f"[bench] ranks share a GPU although {ndev} are visible: {seen}", file=sys.stderr)
                return 4
    group = PeerGroup.from_default(device) if world > 1 else None

    cfg = GPT2Config.preset(a.model)
    cfg.n_ctx = max(cfg.n_ctx, a.seq)
    torch.manual_seed(0)
    model = GPT2(cfg).to(device=device, dtype=torch.bfloat16)
    tcfg = LocalSGDConfig(H=a.H, algo=a.algo)
    trainer = LocalSGDTrainer(model, tcfg, group=group, device=device)

    # synthetic token stream: a pool of distinct batches per peer (different shard per rank)
    g = torch.Generator(device=device)
    g.manual_seed(1000 + rank)
    pool = [torch.randint(0, cfg.vocab_size, (a.batch, a.seq + 1), device=device, generator=g) for _ in range(4)]

    def batch(i):
        b = pool[i % len(pool)]
        return b[:, :-1], b[:, 1:]

    def sync_all():
        if cuda:
            torch.cuda.synchronize()
        if group is not None:
            group.barrier()

    w0 = 0
    graphed = False
    if a.graph and cuda:
        w0 = min(3, a.warmup)
        try:
            trainer.capture(*batch(0), warmup=w0)  # w0 real steps, then hipGraph capture
            graphed = True
        except Exception as e:  # stay correct if capture is refused: eager steps instead
            print(f"[bench] hipGraph capture failed ({type(e).__name__}: {e}); running eager", file=sys.stderr)
            trainer.graph = None
    for i in range(w0, a.warmup):
        trainer.step(*batch(i))
    if group is not None:
        # connect every peer pair of the averaging collective before the timed window (RCCL sets up
        # its point-to-point channels on first use), even when --warmup is shorter than H
        from distributedvolunteercomputing_amd.parallel.collectives import allreduce_sum_

        allreduce_sum_(torch.zeros_like(trainer.delta), group, a.algo)  # same size as the real round
    sync_all()
    trainer.time_reduce = world > 1  # the averaging collective timed apart (algbw / busbw below)
    trainer.reduce_log = []
    t0 = time.perf_counter()
    last = None
    syncs = []
    for i in range(a.steps):
        last = trainer.step(*batch(a.warmup + i))
        if last.synced:
            syncs.append(trainer.last_sync_ms)
    sync_all()
    dt = time.perf_counter() - t0
    # which device each rank ran on, and how many ranks the process group really has
    dev_desc = f"{device.type}:{device.index if device.index is not None else 0}"
    if cuda:
        p = torch.cuda.get_device_properties(device)
        dev_desc += f" {p.name} pci {getattr(p, 'pci_bus_id', '?')}"
    devices = [dev_desc]
    rccl_world = 1
    if world > 1:
        rccl_world = dist.get_world_size()
        devices = [None] * rccl_world
        dist.all_gather_object(devices, dev_desc)
    loss = float(last.extra["loss_t"]) if last is not None else float("nan")
    red = trainer.reduce_log
    red_ms = sum(m for m, _ in red) / len(red) if red else None
    red_bytes = red[0][1] if red else trainer.delta.numel() * trainer.delta.element_size()
    transports = {}
    if world > 1:
        tr = [None] * world
        dist.all_gather_object(tr, _rccl_transports(rccl_log))
        for d in tr:
            for k, v in (d or {}).items():
                transports[k] = transports.get(k, 0) + v
    if group is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    samples = world * a.batch * a.steps
    sps = samples / dt
    tok_s = sps * a.seq
    flops = model.flops_per_token(a.seq) * tok_s
    if rank == 0:
        rec = {
            "metric": "samples/sec GPT-2-small local-SGD",
            "value": round(sps, 3),
            "unit": "samples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(dt / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic (random tokens, random-init weights)",
            "config": {
                "model": a.model,
                "global_batch": world * a.batch,
                "per_peer_batch": a.batch,
                "seq_len": a.seq,
                "parallelism": f"local-sgd dp{world} H={a.H} allreduce={a.algo}",
            },
            "tokens_per_s": round(tok_s, 1),
            "model_tflops_per_gpu": round(flops / world / 1e12, 2),
            "mfu_bf16_dense": round(flops / world / BF16_DENSE_PEAK, 4),
            "final_loss": round(loss, 4),
            "sync_ms": round(trainer.last_sync_ms, 3),
            "sync_ms_timed_mean": round(sum(syncs) / len(syncs), 3) if syncs else None,
            "sync_rounds_timed": len(syncs),
            "rccl_world": rccl_world,
            "backend": dist.get_backend() if world > 1 else None,
            "devices": devices,
            "tuned_gemms": TUNED_GEMMS,
            "hipgraph": graphed,
            # ranks sharing a card (scripts/rccl_rehearsal_launch.py): a functional run, not a per-GPU number
            "ranks_share_gpu": bool(cuda and world > torch.cuda.device_count()),
            # averaging round anatomy (weak scaling: what the collective costs as N grows)
            "avg_bytes_per_rank": red_bytes,
            "avg_collective_ms_mean": round(red_ms, 3) if red_ms else None,
            "avg_algbw_GBps": round(red_bytes / red_ms / 1e6, 4) if red_ms else None,
            "avg_busbw_GBps": round(red_bytes / red_ms / 1e6 * 2 * (world - 1) / world, 4) if red_ms else None,
            "rccl_transports": transports or None,
            "gemm_lt_shapes": sum(1 for v in gemm_choices().values() if v == "lt"),
            "gemm_shapes": len(gemm_choices()),
        }
        line = json.dumps(rec)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
