"""GPT-2 (small / medium / large / xl) for the local-SGD training job.

BASELINE.json configs 2 and 4 (GPT-2-small bf16 local-SGD, GPT-2-medium elastic). There is
no GPT-2 in the reference (its only model is MobileNet-SSD); this is the
north-star training model.

MI355X-first choices:
* bf16 weights/activations, fp32 master weights live in the optimizer (flat buffers);
* every LayerNorm is fused with the residual add that precedes it AND with the bias of the
  GEMM that produced the branch (one HIP kernel reads the residual stream once and writes
  the new residual and the normalised activations; its backward also emits that bias's grad);
* fc bias + tanh-GELU, the token+position embedding, and the vocab-wide softmax
  cross-entropy are HIP kernels; the cross-entropy backward writes the logit gradient in place;
* causal attention (head dim 64) is the HIP flash-attention kernel on the packed qkv layout
  (no permute/cat copies); GEMMs are library GEMMs (hipBLASLt/rocBLAS via TunableOp tables);
* vocabulary padded to a multiple of 128 (50257 -> 50304) so the LM-head GEMM tiles cleanly;
  padded logits are masked inside the loss kernel;
* weight gradients are split-M batched GEMMs reduced by a HIP kernel straight into the flat
  gradient buffer (ops/linear.py).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn.attention import SDPBackend, sdpa_kernel

from .. import ops

# On MI355X the memory-efficient SDPA kernel's backward is 2.1x faster than the flash one at
# the bench shape (B=64, H=12, T=1024, D=64: 1.08 vs 2.25 ms; scripts/attn_bench.py).
_SDPA_BACKENDS = [SDPBackend.EFFICIENT_ATTENTION, SDPBackend.FLASH_ATTENTION, SDPBackend.MATH]


@dataclass
class GPT2Config:
    vocab_size: int = 50257
    padded_vocab: int = 50304
    n_ctx: int = 1024
    n_layer: int = 12
    n_head: int = 12
    n_embd: int = 768
    ln_eps: float = 1e-5

    @staticmethod
    def preset(name: str) -> "GPT2Config":
        table = {
            "gpt2": dict(n_layer=12, n_head=12, n_embd=768),  # 124M
            "gpt2-small": dict(n_layer=12, n_head=12, n_embd=768),
            "gpt2-medium": dict(n_layer=24, n_head=16, n_embd=1024),  # 350M
            "gpt2-large": dict(n_layer=36, n_head=20, n_embd=1280),  # 774M
            "gpt2-xl": dict(n_layer=48, n_head=25, n_embd=1600),  # 1.56B
            "gpt2-tiny": dict(n_layer=2, n_head=2, n_embd=128, n_ctx=128, vocab_size=512, padded_vocab=512),
        }
        return GPT2Config(**table[name])


class Block(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        C = cfg.n_embd
        self.n_head = cfg.n_head
        self.ln1_w = nn.Parameter(torch.ones(C))
        self.ln1_b = nn.Parameter(torch.zeros(C))
        self.attn_w = nn.Parameter(torch.empty(3 * C, C))
        self.attn_b = nn.Parameter(torch.zeros(3 * C))
        self.proj_w = nn.Parameter(torch.empty(C, C))
        self.proj_b = nn.Parameter(torch.zeros(C))
        self.ln2_w = nn.Parameter(torch.ones(C))
        self.ln2_b = nn.Parameter(torch.zeros(C))
        self.fc_w = nn.Parameter(torch.empty(4 * C, C))
        self.fc_b = nn.Parameter(torch.zeros(4 * C))
        self.fc2_w = nn.Parameter(torch.empty(C, 4 * C))
        self.fc2_b = nn.Parameter(torch.zeros(C))

    def attn(self, h):
        B, T, C = h.shape
        H = self.n_head
        # on the native path the QKV bias gradient comes out of the attention backward kernels
        # (column sums of dqkv per block) instead of a separate pass over dqkv
        fuse = (C // H == 64 and h.dtype == torch.bfloat16 and ops.native_linear_ok(self.attn_w)
                and self.attn_b.requires_grad)
        qkv = ops.linear(h, self.attn_w, self.attn_b, bias_grad_elsewhere=fuse).view(B, T, 3, H, C // H)
        if C // H == 64 and qkv.is_cuda:
            y = ops.causal_attention(qkv, bias=self.attn_b if fuse else None)  # HIP flash attention, packed layout
        else:
            q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)
            with sdpa_kernel(_SDPA_BACKENDS):
                y = F.scaled_dot_product_attention(q, k, v, is_causal=True)
            y = y.transpose(1, 2)
        # no bias here: proj_b is added (and its gradient reduced) by the following fused
        # residual-add + LayerNorm kernel
        return ops.linear(y.reshape(B, T, C), self.proj_w)

    def mlp(self, h):
        # fc bias + GELU in the fc GEMM's epilogue (and gelu' + bias grad in the backward GEMM's),
        # fc2 bias fused into the next add+LayerNorm
        return ops.mlp_gelu(h, self.fc_w, self.fc_b, self.fc2_w)


class GPT2(nn.Module):
    def __init__(self, cfg: GPT2Config):
        super().__init__()
        self.cfg = cfg
        C = cfg.n_embd
        self.wte = nn.Parameter(torch.empty(cfg.padded_vocab, C))
        self.wpe = nn.Parameter(torch.empty(cfg.n_ctx, C))
        self.blocks = nn.ModuleList([Block(cfg) for _ in range(cfg.n_layer)])
        self.lnf_w = nn.Parameter(torch.ones(C))
        self.lnf_b = nn.Parameter(torch.zeros(C))
        self.reset_parameters()

    @torch.no_grad()
    def reset_parameters(self, seed: int | None = None):
        g = torch.Generator(device="cpu")
        g.manual_seed(1234 if seed is None else seed)
        std = 0.02
        proj_std = 0.02 / math.sqrt(2 * self.cfg.n_layer)

        def init(p, s):
            p.copy_(torch.randn(p.shape, generator=g) * s)

        init(self.wte, std)
        init(self.wpe, 0.01)
        for b in self.blocks:
            init(b.attn_w, std)
            init(b.proj_w, proj_std)
            init(b.fc_w, std)
            init(b.fc2_w, proj_std)

    def num_params(self, non_embedding=True):
        n = sum(p.numel() for p in self.parameters())
        if non_embedding:
            n -= self.wpe.numel()
        return n

    def flops_per_token(self, T: int) -> float:
        """Training FLOPs/token: 6*N (dense) + 12*L*C*T (attention, fwd+bwd, causal not halved)."""
        c = self.cfg
        N = self.num_params(non_embedding=True)
        return 6.0 * N + 12.0 * c.n_layer * c.n_embd * T

    def forward(self, idx, targets=None):
        B, T = idx.shape
        cfg = self.cfg
        x = ops.embed(idx, self.wte, self.wpe)  # fused token + position gather (HIP)
        eps = cfg.ln_eps
        blocks = self.blocks
        h, resid = ops.add_layernorm(x, None, blocks[0].ln1_w, blocks[0].ln1_b, eps)
        for i, blk in enumerate(blocks):
            a = blk.attn(h)
            h, resid = ops.add_layernorm(resid, a, blk.ln2_w, blk.ln2_b, eps, branch_bias=blk.proj_b)
            m = blk.mlp(h)
            if i + 1 < len(blocks):
                nxt = blocks[i + 1]
                h, resid = ops.add_layernorm(resid, m, nxt.ln1_w, nxt.ln1_b, eps, branch_bias=blk.fc2_b)
            else:
                h, resid = ops.add_layernorm(resid, m, self.lnf_w, self.lnf_b, eps, branch_bias=blk.fc2_b)
        if targets is None:
            return ops.linear(h, self.wte)[..., : cfg.vocab_size]  # tied LM head, [B, T, Vp]
        return ops.lm_head_cross_entropy(h, self.wte, targets, cfg.vocab_size)
