#!/usr/bin/env python3
"""Per-config throughput of the BASELINE.json training configs on ONE MI355X peer.

Config 2 (GPT-2-small local-SGD) is bench.py. Here, on a single GPU (the multi-peer
collective is then a no-op, everything else — compression kernels, sharded optimizer,
fused AdamW — runs in full):
  3: ResNet-50, synthetic ImageNet, local-SGD H=4 + top-k (1%) error-feedback compression
  4: GPT-2-medium local-SGD H=4
  5: Llama-3-8B sharded-optimizer trainer + PowerSGD rank 4 (HBM sizing check on 288 GB)
Prints one JSON line per config. Under a torchrun-style env (WORLD_SIZE > 1) config 5 runs one
sharded peer per rank (ZeRO-1 over the group, PowerSGD-averaged gradients, parameter all-gather).
On one process (no WORLD_SIZE > 1) several configs run one child process each, started before this
parent touches the GPU: run in one process after config 3, config 4 measured 323-357 samples/s
against 400-401 on its own (gpurun_out/c4ord*, profiles/r6_final_validation.txt), whatever config 3's
convolution path -- a process-state interaction (allocator / library state left by the ResNet), not
a property of config 4's step. BENCH_CONFIGS_INPROC=1 keeps them in one process.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

from distributedvolunteercomputing_amd.utils.tuning import enable_tuned_gemms

enable_tuned_gemms(int(os.environ.get("LOCAL_RANK", "0")))

import torch  # noqa: E402


def _time(step, warmup, steps):
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps, out


def _graph(tr, x, y, a):
    """hipGraph capture of the local step (bench.py's path: zero-grad + forward + backward + fused AdamW replayed
    as one graph launch; the averaging round stays outside); eager steps if capture is refused."""
    if a.no_graph:
        return False
    try:
        tr.capture(x, y, warmup=3)
        return True
    except Exception as e:  # stay correct: eager steps instead
        print(f"[bench_configs] hipGraph capture failed ({type(e).__name__}: {e}); running eager", file=sys.stderr)
        tr.graph = None
        return False


def cfg3(a, dev):
    from distributedvolunteercomputing_amd.models.resnet import enable_conv_find, resnet50
    from distributedvolunteercomputing_amd.parallel.compression import TopKCompressor
    from distributedvolunteercomputing_amd.parallel.local_sgd import LocalSGDConfig, LocalSGDTrainer

    m = resnet50().to(dev, torch.bfloat16).to(memory_format=torch.channels_last)
    enable_conv_find()
    tr = LocalSGDTrainer(m, LocalSGDConfig(H=4, lr=1e-3, weight_decay=0.0), device=dev)
    tr.compressor = TopKCompressor(tr.flat.numel, 0.01, dev)
    B = a.resnet_batch
    x = torch.randn(B, 3, 224, 224, device=dev).to(torch.bfloat16).to(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (B,), device=dev)
    graphed = _graph(tr, x, y, a)
    dt, st = _time(lambda: tr.step(x, y), 4, a.steps)
    # cost of one compressed averaging round on its own (warmed up: the first call loads the
    # compression kernels' code objects; mean of 10 rounds)
    for _ in range(2):
        tr.compressor.allreduce_mean(tr.delta, None)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        tr.compressor.allreduce_mean(tr.delta, None)
    torch.cuda.synchronize()
    return {"config": 3, "model": "resnet50", "images_per_s": round(B / dt, 1), "ms_per_step": round(dt * 1e3, 2),
            "batch": B, "topk_ratio": 0.01, "topk_round_ms": round((time.perf_counter() - t0) * 1e3 / 10, 3),
            "params": tr.flat.numel, "hipgraph": graphed}


def cfg4(a, dev):
    from distributedvolunteercomputing_amd.models.gpt2 import GPT2, GPT2Config
    from distributedvolunteercomputing_amd.parallel.local_sgd import LocalSGDConfig, LocalSGDTrainer

    cfg = GPT2Config.preset("gpt2-medium")
    m = GPT2(cfg).to(dev, torch.bfloat16)
    tr = LocalSGDTrainer(m, LocalSGDConfig(H=4), device=dev)
    B, T = a.medium_batch, 1024
    x = torch.randint(0, cfg.vocab_size, (B, T + 1), device=dev)
    xi, yi = x[:, :-1].contiguous(), x[:, 1:].contiguous()
    graphed = _graph(tr, xi, yi, a)
    dt, _ = _time(lambda: tr.step(xi, yi), 4, a.steps)
    return {"config": 4, "model": "gpt2-medium", "samples_per_s": round(B / dt, 2), "tokens_per_s": round(B * T / dt),
            "ms_per_step": round(dt * 1e3, 2), "batch": B, "mfu_bf16_dense": round(m.flops_per_token(T) * B * T / dt /
                                                                                    2.5e15, 4), "hipgraph": graphed}


def cfg5(a, dev):
    from distributedvolunteercomputing_amd.models.llama import Llama, LlamaConfig
    from distributedvolunteercomputing_amd.parallel.compression import PowerSGDCompressor
    from distributedvolunteercomputing_amd.parallel.zero import ShardedConfig, ShardedDPTrainer

    name = a.llama
    cfg = LlamaConfig.preset(name)
    with torch.device("meta"):
        m = Llama(cfg, init=False)
    m = m.to_empty(device=dev).to(torch.bfloat16)
    with torch.no_grad():
        for p in m.parameters():
            p.normal_(0.0, 0.02) if p.dim() >= 2 else p.fill_(1.0)
    torch.cuda.reset_peak_memory_stats()
    group = None
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:  # one sharded peer per rank (torchrun-style env)
        import torch.distributed as dist

        from distributedvolunteercomputing_amd.parallel.peer_group import PeerGroup

        if not dist.is_initialized():
            dist.init_process_group("nccl", device_id=dev)
        group = PeerGroup.from_default(dev)
    reps = min(a.llama_replicas, group.size - 1) if group is not None else 0
    tr = ShardedDPTrainer(m, ShardedConfig(lr=1e-4, replicas=max(reps, 1), replicate=reps > 0), group=group,
                          device=dev)
    tr.compressor = PowerSGDCompressor(tr.flat, rank=4, device=dev)
    B, T = a.llama_batch, a.llama_seq
    x = torch.randint(0, cfg.vocab_size, (B, T + 1), device=dev)
    dt, loss = _time(lambda: tr.step(x[:, :-1], x[:, 1:]), 2, max(2, a.steps // 2))
    peers = group.size if group is not None else 1
    return {"config": 5, "model": name, "params": m.num_params(), "peers": peers, "replicas": reps,
            "tokens_per_s": round(B * T / dt, 1),
            "ms_per_step": round(dt * 1e3, 1), "batch": B, "seq": T, "loss": round(float(loss), 3),
            "peak_hbm_gb": round(torch.cuda.max_memory_allocated() / 2**30, 1),
            "powersgd_compression_ratio": round(tr.compressor.compression_ratio, 1),
            "mfu_bf16_dense": round(m.flops_per_token(T) * B * T / dt / 2.5e15, 4)}


def child_argv(argv, config):
    """argv for the child process of one config: the parent's arguments with --configs replaced."""
    rest, skip = [], False
    for arg in argv:
        if skip:
            skip = False
        elif arg == "--configs":
            skip = True
        elif not arg.startswith("--configs="):
            rest.append(arg)
    return ["--configs", config] + rest


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="3,4,5")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--resnet-batch", type=int, default=128)
    ap.add_argument("--medium-batch", type=int, default=32)
    ap.add_argument("--llama", default="llama3-8b")
    ap.add_argument("--llama-batch", type=int, default=2)
    ap.add_argument("--llama-seq", type=int, default=2048)
    ap.add_argument("--no-graph", action="store_true", help="configs 3 / 4: eager steps (no hipGraph capture)")
    ap.add_argument("--llama-replicas", type=int, default=2, help="config 5 with several peers: shard replicas")
    a = ap.parse_args()
    configs = a.configs.split(",")
    if len(configs) > 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1 and os.environ.get("BENCH_CONFIGS_INPROC") != "1":
        # one child per config; this parent never initialises the GPU
        rc = 0
        for c in configs:
            rc = max(rc, subprocess.run([sys.executable, os.path.abspath(__file__)] + child_argv(sys.argv[1:], c)).returncode)
        return rc
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    fns = {"3": cfg3, "4": cfg4, "5": cfg5}
    rc = 0
    for c in configs:
        try:
            rec = fns[c](a, dev)
        except Exception as e:  # report and continue with the next config
            rec = {"config": int(c), "error": repr(e)[:500]}
            print(f"[bench_configs rank {os.environ.get('RANK', '0')}] config {c} failed: {e!r}", file=sys.stderr,
                  flush=True)
            rc = 1
        if int(os.environ.get("RANK", "0")) == 0:
            print(json.dumps(rec), flush=True)
        torch.cuda.empty_cache()
    return rc


if __name__ == "__main__":
    sys.exit(main())
