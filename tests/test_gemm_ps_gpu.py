"""Persistent store-overlapped GEMM (csrc/kernels/gemm_ps.hip) against an fp32 PyTorch reference:
every epilogue, one tile per workgroup, several tiles per workgroup (the continuous LDS ring across
tile boundaries and the stores left in flight into the next tile), a reduced grid, strided rows."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N,K,cap", [(256, 256, 256, 0), (2048, 3072, 768, 0), (4096, 2304, 768, 16),
                                       (8192, 768, 3072, 8), (256 * 40, 512, 1024, 0)])
def test_gemm_ps_matches_fp32(gpu, M, N, K, cap):
    from distributedvolunteercomputing_amd.ops import native

    C = native()
    torch.manual_seed(M + N + K)
    dev = "cuda"
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05
    bias = torch.randn(N, device=dev, dtype=torch.bfloat16) * 0.1
    ref = a.float() @ b.float().t()
    for epi in range(3):
        c = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
        c2 = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
        C.gemm_ps(a, b, c, c2, bias, None, epi, cap)
        torch.cuda.synchronize()
        want = ref if epi == 0 else ref + bias.float()
        err = (c.float() - want).abs().max().item()
        assert err < 2e-2 * want.abs().max().item(), (epi, err)
        if epi == 2:
            g = F.gelu(want, approximate="tanh")
            assert (c2.float() - g).abs().max().item() < 3e-2 * g.abs().max().item()
    # DGELU: c = (a b^T) * gelu'(pre) and fp32 column sums (the bias gradient) into cs
    pre = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    c = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
    cs = torch.zeros(N, device=dev, dtype=torch.float32)
    C.gemm_ps(a, b, c, pre, None, cs, 4, cap)
    torch.cuda.synchronize()
    x = pre.float().requires_grad_()
    F.gelu(x, approximate="tanh").backward(ref.to(torch.bfloat16).float())
    assert (c.float() - x.grad).abs().max().item() < 2e-2 * x.grad.abs().max().item()
    s = x.grad.sum(0)
    assert (cs - s).abs().max().item() < 1e-2 * s.abs().max().item() + 1e-2
    # round 6 pair: epilogue 5 (c = gelu'(pre), c2 = gelu(pre), pre = a b^T + bias) and epilogue 6
    # (c = (a b^T) * c2 with fp32 column sums): the fused MLP's forward and fc2 input gradient
    gp = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
    act = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
    C.gemm_ps(a, b, gp, act, bias, None, 5, cap)
    torch.cuda.synchronize()
    pre32 = (ref + bias.float()).to(torch.bfloat16).float().requires_grad_()  # the kernel rounds pre to bf16
    g = F.gelu(pre32, approximate="tanh")
    assert (act.float() - g.detach()).abs().max().item() < 3e-2 * g.abs().max().item()
    g.backward(torch.ones_like(g))
    assert (gp.float() - pre32.grad).abs().max().item() < 1e-2  # gelu' lies in [-0.17, 1.13]
    c = torch.full((M, N), float("nan"), device=dev, dtype=torch.bfloat16)
    cs = torch.zeros(N, device=dev, dtype=torch.float32)
    C.gemm_ps(a, b, c, gp, None, cs, 6, cap)
    torch.cuda.synchronize()
    want = ref.to(torch.bfloat16).float() * pre32.grad
    assert (c.float() - want).abs().max().item() < 2e-2 * want.abs().max().item()
    s = want.sum(0)
    assert (cs - s).abs().max().item() < 1e-2 * s.abs().max().item() + 1e-2


def test_gemm_ps_strided_rows_and_refusals(gpu):
    from distributedvolunteercomputing_amd.ops import native

    C = native()
    dev = "cuda"
    a = torch.randn(512, 1024, device=dev, dtype=torch.bfloat16)[:, :768]  # lda = 1024
    b = torch.randn(768, 768, device=dev, dtype=torch.bfloat16) * 0.05
    wide = torch.zeros(512, 1024, device=dev, dtype=torch.bfloat16)
    c = wide[:, :768]  # ldc = 1024; columns past 768 must stay untouched
    C.gemm_ps(a, b, c)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().t()
    assert (c.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()
    assert wide[:, 768:].abs().max().item() == 0
    assert not C.gemm_ps_supported(512, 768, 192, 0)  # K % 128
    assert not C.gemm_ps_supported(500, 768, 768, 0)  # M % 256
    with pytest.raises(RuntimeError):
        C.gemm_ps(a[:, 4:260], b[:256, :256].contiguous(), torch.empty(512, 256, device=dev, dtype=torch.bfloat16))


def test_gemm_ps_refuses_unknown_epilogues(gpu):
    """Only the real epilogues are accepted: 3 (gemm_nt's DGELU code) and the removed no-store
    diagnostic 7 are refused (5 and 6 are the round-6 gelu'-in-the-forward pair)."""
    from distributedvolunteercomputing_amd.ops import native

    C = native()
    for epi in (3, 7, 8):
        assert not C.gemm_ps_supported(512, 256, 768, epi)
    for epi in (5, 6):
        assert C.gemm_ps_supported(512, 256, 768, epi)
    a = torch.randn(512, 768, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(256, 768, device="cuda", dtype=torch.bfloat16)
    c = torch.empty(512, 256, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        C.gemm_ps(a, b, c, None, None, None, 7)


def test_gemm_ps_repeat_runs_bit_identical(gpu):
    """The fused-MLP launches are deterministic (no atomics in the outputs): repeats must reproduce
    the first run bit for bit — a slot read before its DMA landed would show as differing tiles
    (scripts/gemm_ps_stress.py runs the full-size version)."""
    from distributedvolunteercomputing_amd.ops import native

    C = native()
    torch.manual_seed(3)
    M, N, K = 16384, 3072, 768
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.03
    b = torch.randn(N, device="cuda", dtype=torch.bfloat16) * 0.1
    pre, act = torch.empty(M, N, device="cuda", dtype=torch.bfloat16), torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    C.gemm_ps(x, w, pre, act, b, None, 2)
    g_pre, g_act = pre.clone(), act.clone()
    d, cs = torch.empty_like(pre), torch.zeros(N, device="cuda")
    C.gemm_ps(x, w, d, g_pre, None, cs, 4)
    g_d = d.clone()
    for _ in range(20):
        C.gemm_ps(x, w, pre, act, b, None, 2)
        C.gemm_ps(x, w, d, g_pre, None, cs, 4)
        assert torch.equal(pre, g_pre) and torch.equal(act, g_act) and torch.equal(d, g_d)
