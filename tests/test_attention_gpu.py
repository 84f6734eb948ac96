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


@pytest.mark.parametrize("B,T,H", [(2, 200, 3), (1, 1024, 12), (3, 77, 2)])
@pytest.mark.parametrize("preset", [False, True])
def test_attention_fused_qkv_bias_grad(gpu, B, T, H, preset):
    """linear(..., bias_grad_elsewhere=True) + causal_attention(qkv, bias=b): the bias gradient is
    reduced from the backward kernels' per-block column sums (T not a multiple of 128: padded
    query/key rows must not contribute) and equals the column sums of dqkv."""
    torch.manual_seed(2)
    C = H * 64
    x = torch.randn(B, T, C, device=gpu).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(3 * C, C, device=gpu) * C ** -0.5).to(torch.bfloat16).requires_grad_()
    b = (torch.randn(3 * C, device=gpu) * 0.1).to(torch.bfloat16).requires_grad_()
    if preset:  # flat-buffer style: the gradient is added into the existing .grad
        b.grad = torch.full_like(b, 0.5)
    qkv = ops.linear(x, w, b, bias_grad_elsewhere=True).view(B, T, 3, H, 64)
    qkv.retain_grad()
    out = ops.causal_attention(qkv, bias=b)
    do = torch.randn_like(out)
    (out.float() * do.float()).sum().backward()
    ref = qkv.grad.float().reshape(-1, 3 * C).sum(0) + (0.5 if preset else 0.0)
    rel = (b.grad.float() - ref).norm() / ref.norm()
    assert rel < 1e-2, float(rel)


def test_attention_matches_sdpa_at_bench_shape(gpu):
    torch.manual_seed(1)
    B, T, H = 4, 1024, 12
    qkv = torch.randn(B, T, 3, H, 64, device=gpu).to(torch.bfloat16)
    out = ops.causal_attention(qkv)
    q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)
    ref = torch.nn.functional.scaled_dot_product_attention(q, k, v, is_causal=True).transpose(1, 2)
    rel = (out.float() - ref.float()).norm() / ref.float().norm()
    assert rel < 1e-2, float(rel)


DEFAULT_VARIANT = (3, 2, 12, 1)  # csrc/kernels/attention.hip g_fwd_wpe, g_fwd_dma, g_bwd_dma, g_stage_epi


@pytest.mark.parametrize("variant", [(2, 0, 0, 0), (3, 0, 3, 1), (2, 1, 2, 1), (3, 1, 1, 0), (3, 1, 1, 1),
                                     (2, 2, 4, 1), (3, 2, 8, 1), DEFAULT_VARIANT])
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
        C.attn_set_variant(*DEFAULT_VARIANT)  # the defaults, for the tests that run after this one


def _ref_gqa32(q, k, v, scale):
    rep = q.shape[1] // k.shape[1]
    k = k.repeat_interleave(rep, dim=1)
    v = v.repeat_interleave(rep, dim=1)
    T = q.shape[2]
    s = (q @ k.transpose(-1, -2)) * scale
    mask = torch.triu(torch.ones(T, T, dtype=torch.bool, device=q.device), 1)
    p = torch.softmax(s.masked_fill(mask, float("-inf")), -1)
    return (p @ v).transpose(1, 2)  # [B, T, Hq, D]


@pytest.mark.parametrize("B,Hq,Hkv,T,D", [(2, 4, 2, 200, 128), (1, 8, 2, 1024, 128), (2, 4, 4, 77, 64),
                                          (1, 32, 8, 256, 128), (1, 6, 1, 130, 64)])
def test_gqa_attention_fwd_bwd(gpu, B, Hq, Hkv, T, D):
    """Head-major GQA flash attention (Llama layout, attention_hm.hip) vs an fp32 reference:
    output [B, T, Hq, D] and the gradients of q, k, v (k/v summed over each group's query heads)."""
    torch.manual_seed(3)
    q = torch.randn(B, Hq, T, D, device=gpu).to(torch.bfloat16).requires_grad_()
    k = torch.randn(B, Hkv, T, D, device=gpu).to(torch.bfloat16).requires_grad_()
    v = torch.randn(B, Hkv, T, D, device=gpu).to(torch.bfloat16).requires_grad_()
    scale = 1 / math.sqrt(D)
    out = ops.gqa_attention(q, k, v)
    assert out.shape == (B, T, Hq, D)
    q32, k32, v32 = (t.detach().float().requires_grad_() for t in (q, k, v))
    ref = _ref_gqa32(q32, k32, v32, scale)
    err = (out.float() - ref).abs().max().item()
    assert err < 2e-2, err
    do = torch.randn_like(ref).to(torch.bfloat16).float()
    (out.float() * do).sum().backward()
    (ref * do).sum().backward()
    for nm, a, r in (("q", q.grad, q32.grad), ("k", k.grad, k32.grad), ("v", v.grad, v32.grad)):
        rel = (a.float() - r).norm() / (r.norm() + 1e-6)
        assert rel < 2e-2, (nm, float(rel))


def test_gqa_attention_dkv_split_variant(gpu):
    """D = 128 backward with dK and dV as two launches (the non-default variant) matches the
    default single-launch kernel."""
    C = ops.native()
    torch.manual_seed(8)
    q = torch.randn(1, 8, 300, 128, device=gpu).to(torch.bfloat16)
    k = torch.randn(1, 2, 300, 128, device=gpu).to(torch.bfloat16)
    v = torch.randn(1, 2, 300, 128, device=gpu).to(torch.bfloat16)
    o, lse = C.attn_hm_fwd(q, k, v, 128 ** -0.5)
    do = torch.randn_like(o)
    g_fused = C.attn_hm_bwd(q, k, v, o, do, lse, 128 ** -0.5)
    C.attn_hm_set_variant(1)
    try:
        g_split = C.attn_hm_bwd(q, k, v, o, do, lse, 128 ** -0.5)
    finally:
        C.attn_hm_set_variant(0)
    for a, b in zip(g_fused, g_split):
        assert (a.float() - b.float()).abs().max().item() < 1e-2


def test_gqa_attention_deterministic(gpu):
    C = ops.native()
    torch.manual_seed(6)
    q = torch.randn(2, 8, 512, 128, device=gpu).to(torch.bfloat16)
    k = torch.randn(2, 2, 512, 128, device=gpu).to(torch.bfloat16)
    v = torch.randn(2, 2, 512, 128, device=gpu).to(torch.bfloat16)
    outs = [C.attn_hm_fwd(q, k, v, 128 ** -0.5) for _ in range(3)]
    for o, l in outs[1:]:
        assert torch.equal(o, outs[0][0]) and torch.equal(l, outs[0][1])
    do = torch.randn_like(outs[0][0])
    gs = [C.attn_hm_bwd(q, k, v, outs[0][0], do, outs[0][1], 128 ** -0.5) for _ in range(3)]
    for g in gs[1:]:
        assert all(torch.equal(a, b) for a, b in zip(g, gs[0]))
