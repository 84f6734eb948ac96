"""Llama-3 family (BASELINE.json config 5: "Llama-3-8B, optimizer-state shard across 8
volunteer peers (288 GB HBM per GPU sizing), PowerSGD rank-4 compression").

RMSNorm (with the residual add fused), SwiGLU and the rotary embedding (fused with the QKV split
into head-major q/k/v, ops/rope.py) are HIP kernels; GEMMs are library GEMMs; attention (head dim
128, grouped-query) is the head-major GQA flash attention of attention_hm.hip (ops.gqa_attention),
which writes its output token-major for the o-projection.

Memory sizing for 8B on one MI355X peer (288 GB HBM): bf16 params 16 GB + bf16 grads 16 GB,
plus fp32 master/m/v = 96 GB for the whole model -> 12 GB per peer when sharded over 8
(24 GB with the buddy replica kept for fault tolerance), leaving > 200 GB for activations.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn

from .. import ops


@dataclass
class LlamaConfig:
    vocab_size: int = 128256
    dim: int = 4096
    n_layers: int = 32
    n_heads: int = 32
    n_kv_heads: int = 8
    ffn_dim: int = 14336
    rope_theta: float = 500000.0
    norm_eps: float = 1e-5
    max_seq: int = 8192

    @staticmethod
    def preset(name: str) -> "LlamaConfig":
        t = {
            "llama3-8b": dict(),
            "llama3.2-1b": dict(dim=2048, n_layers=16, n_heads=32, n_kv_heads=8, ffn_dim=8192),
            "llama3.2-3b": dict(dim=3072, n_layers=28, n_heads=24, n_kv_heads=8, ffn_dim=8192),
            "llama-tiny": dict(vocab_size=512, dim=128, n_layers=2, n_heads=4, n_kv_heads=2, ffn_dim=256, max_seq=256),
        }
        return LlamaConfig(**t[name])


from ..ops.rope import apply_rope, rope_tables  # noqa: E402,F401  (re-exported for callers)

class LlamaBlock(nn.Module):
    def __init__(self, c: LlamaConfig):
        super().__init__()
        self.c = c
        hd = c.dim // c.n_heads
        self.attn_norm = nn.Parameter(torch.ones(c.dim))
        self.wqkv = nn.Parameter(torch.empty((c.n_heads + 2 * c.n_kv_heads) * hd, c.dim))
        self.wo = nn.Parameter(torch.empty(c.dim, c.dim))
        self.ffn_norm = nn.Parameter(torch.ones(c.dim))
        self.w13 = nn.Parameter(torch.empty(2 * c.ffn_dim, c.dim))  # [gate | up]
        self.w2 = nn.Parameter(torch.empty(c.dim, c.ffn_dim))

    def attn(self, h, cos, sin):
        c = self.c
        B, T, D = h.shape
        # fused QKV projection -> one HIP kernel: split, rotary embedding on q/k, head-major q/k/v
        q, k, v = ops.rope_qkv(ops.linear(h, self.wqkv), cos, sin, c.n_heads, c.n_kv_heads)
        y = ops.gqa_attention(q, k, v)  # HIP flash attention (GQA, head-major in, token-major out)
        return ops.linear(y.reshape(B, T, D), self.wo)

    def mlp(self, h):
        return ops.linear(ops.swiglu(ops.linear(h, self.w13)), self.w2)


class Llama(nn.Module):
    def __init__(self, c: LlamaConfig, seed: int = 0, init: bool = True):
        super().__init__()
        self.c = c
        self.tok = nn.Parameter(torch.empty(c.vocab_size, c.dim))
        self.layers = nn.ModuleList([LlamaBlock(c) for _ in range(c.n_layers)])
        self.norm = nn.Parameter(torch.ones(c.dim))
        self.out = nn.Parameter(torch.empty(c.vocab_size, c.dim))
        if init:
            self.reset_parameters(seed)

    @torch.no_grad()
    def reset_parameters(self, seed=0):
        g = torch.Generator(device=self.tok.device if self.tok.device.type == "cpu" else "cpu").manual_seed(seed)
        std = 0.02
        for n, p in self.named_parameters():
            if p.dim() >= 2:
                s = std / math.sqrt(2 * self.c.n_layers) if n.endswith(("wo", "w2")) else std
                p.copy_(torch.randn(p.shape, generator=g) * s)

    def num_params(self):
        return sum(p.numel() for p in self.parameters())

    def flops_per_token(self, T):
        c = self.c
        return 6.0 * (self.num_params() - self.tok.numel()) + 12.0 * c.n_layers * c.dim * T

    def forward(self, idx, targets=None):
        B, T = idx.shape
        c = self.c
        cos, sin = rope_tables(T, c.dim // c.n_heads, c.rope_theta, idx.device)
        x = ops.embed(idx, self.tok)
        h, resid = ops.add_rmsnorm(x, None, self.layers[0].attn_norm, c.norm_eps)
        for i, L in enumerate(self.layers):
            a = L.attn(h, cos, sin)
            h, resid = ops.add_rmsnorm(resid, a, L.ffn_norm, c.norm_eps)
            m = L.mlp(h)
            nw = self.layers[i + 1].attn_norm if i + 1 < len(self.layers) else self.norm
            h, resid = ops.add_rmsnorm(resid, m, nw, c.norm_eps)
        logits = ops.linear(h, self.out)
        if targets is None:
            return logits
        return ops.cross_entropy(logits.view(B * T, -1), targets.reshape(-1), vocab=c.vocab_size)
