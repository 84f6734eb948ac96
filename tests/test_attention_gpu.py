"""HIP flash attention (head dim 64, causal, packed qkv) vs fp32 PyTorch reference."""
import math

import pytest
import torch

from distributedvolunteercomputing_amd import ops

pytestmark = pytest.mark.gpu


def _ref(qkv32, scale):
    q, k, v = qkv32.permute(2, 0, 3, 1, 4).unbind(0)
    T = q.shape[2]
    s = (q @ k.transpose(-1, -2)) * scale
    mask = torch.triu(torch.ones(T, T, dtype=torch.bool, device=q.device), 1)
    s = s.masked_fill(mask, float("-inf"))
    p = torch.softmax(s, -1)
    return (p @ v).transpose(1, 2)  # [B, T, H, D]


@pytest.mark.parametrize("B,T,H", [(2, 128, 2), (1, 1024, 3), (2, 200, 2), (1, 64, 1), (3, 77, 2)])
def test_attention_fwd_bwd(gpu, B, T, H):
    torch.manual_seed(0)
    qkv = torch.randn(B, T, 3, H, 64, device=gpu).to(torch.bfloat16).requires_grad_()
    scale = 1 / math.sqrt(64)
    out = ops.causal_attention(qkv)
    q32 = qkv.detach().float().requires_grad_()
    ref = _ref(q32, scale)
    err = (out.float() - ref).abs().max().item()
    assert err < 2e-2, err
    do = torch.randn_like(ref)
    (out.float() * do).sum().backward()
    (ref * do).sum().backward()
    g, gr = qkv.grad.float(), q32.grad
    for i, nm in enumerate("qkv"):
        a, r = g[:, :, i], gr[:, :, i]
        rel = (a - r).norm() / (r.norm() + 1e-6)
        assert rel < 2e-2, (nm, float(rel))


def test_attention_matches_sdpa_at_bench_shape(gpu):
    torch.manual_seed(1)
    B, T, H = 4, 1024, 12
    qkv = torch.randn(B, T, 3, H, 64, device=gpu).to(torch.bfloat16)
    out = ops.causal_attention(qkv)
    q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)
    ref = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2)
    rel = (out.float() - ref.float()).norm() / ref.float().norm()
    assert rel < 1e-2, float(rel)


@pytest.mark.parametrize("variant", [(2, 0, 0), (3, 0, 3), (2, 1, 2), (3, 1, 1)])
def test_attention_deterministic(gpu, variant):
    """Same inputs, same kernel -> bitwise identical outputs (a race on the double-buffered LDS
    tiles would show up here as run-to-run differences)."""
    C = ops.native()
    torch.manual_seed(5)
    B, T, H = 8, 1024, 12
    qkv = torch.randn(B, T, 3, H, 64, device=gpu).to(torch.bfloat16)
    C.attn_set_variant(*variant)
    try:
        outs = [C.attn_fwd(qkv, 0.125) for _ in range(4)]
        torch.cuda.synchronize()
        for o, l in outs[1:]:
            nd = int((o != outs[0][0]).sum())
            assert nd == 0, f"{nd} output elements differ between identical launches"
            assert torch.equal(l, outs[0][1])
        dO = torch.randn_like(outs[0][0])
        gs = [C.attn_bwd(qkv, outs[0][0], dO, outs[0][1], 0.125) for _ in range(3)]
        for g in gs[1:]:
            assert torch.equal(g, gs[0])
    finally:
        C.attn_set_variant(3, 1, 1)
