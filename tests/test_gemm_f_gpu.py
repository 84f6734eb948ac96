"""Forward GEMM in the library's geometry (csrc/kernels/gemm_f.hip: 256 x 256 tiles, 4 waves of 128 x 128 or 8 of 128 x 64)
against an fp32 PyTorch reference: one tile, many tiles, a 128-column last panel, the shortest K (3 slices ahead of 6), ragged M (rows past
the operand read as zeros and are never stored), strided rows, refusals, and bit-identical repeats."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("waves", [4, 8])
@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (4096, 2304, 768), (8192, 768, 3072), (300, 512, 192),
                                   (1000, 256, 1024), (256 * 33, 768, 768),
                                   (700, 640, 384), (512, 128, 256)])
def test_gemm_f_matches_fp32(gpu, M, N, K, waves):
    from distributedvolunteercomputing_amd.ops import native

    C = native()
    torch.manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.05
    full = torch.full((M + 7, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    c = full[:M]
    C.gemm_f(a, b, c, None, waves)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().t()
    err = (c.float() - ref).abs().max().item()
    assert err < 1e-2 * ref.abs().max().item(), err
    assert torch.isnan(full[M:].float()).all()  # nothing stored past row M
    bias = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    C.gemm_f(a, b, c, bias, waves)
    torch.cuda.synchronize()
    ref = ref + bias.float()
    assert (c.float() - ref).abs().max().item() < 1e-2 * ref.abs().max().item()


def test_gemm_f_strided_rows_and_refusals(gpu):
    from distributedvolunteercomputing_amd.ops import native

    C = native()
    a = torch.randn(512, 1024, device="cuda", dtype=torch.bfloat16)[:, :768]  # lda = 1024
    b = torch.randn(1280, 768, device="cuda", dtype=torch.bfloat16)[:512] * 0.05
    wide = torch.zeros(512, 1024, device="cuda", dtype=torch.bfloat16)
    c = wide[:, :512]  # ldc = 1024; columns past 512 must stay untouched
    C.gemm_f(a, b, c)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().t()
    assert (c.float() - ref).abs().max().item() < 1e-2 * ref.abs().max().item()
    assert wide[:, 512:].abs().max().item() == 0
    assert not C.gemm_f_supported(512, 768, 128)  # K < 192
    assert not C.gemm_f_supported(512, 768, 800)  # K % 64
    assert not C.gemm_f_supported(512, 704, 768)  # N % 128
    with pytest.raises(RuntimeError):
        C.gemm_f(a, b[:, :512].contiguous(), torch.empty(512, 512, device="cuda", dtype=torch.bfloat16))


def test_gemm_f_repeat_runs_bit_identical(gpu):
    """A slot read before its DMA landed would show as differing tiles between repeats."""
    from distributedvolunteercomputing_amd.ops import native

    C = native()
    torch.manual_seed(5)
    x = torch.randn(16384, 768, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(2304, 768, device="cuda", dtype=torch.bfloat16) * 0.03
    y = torch.empty(16384, 2304, device="cuda", dtype=torch.bfloat16)
    for waves in (4, 8):
        C.gemm_f(x, w, y, None, waves)
        g = y.clone()
        for _ in range(20):
            C.gemm_f(x, w, y, None, waves)
            assert torch.equal(y, g)


def test_linear_on_gemm_f_matches_library(gpu):
    """config.gemm_fwd = "vcx" routes the linear layer's forward (with bias) and its input gradient through
    gemm_f; both match the library path."""
    from distributedvolunteercomputing_amd import config, ops

    torch.manual_seed(7)
    x = torch.randn(4, 256, 384, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(640, 384, device="cuda", dtype=torch.bfloat16) * 0.05).requires_grad_()
    b = (torch.randn(640, device="cuda", dtype=torch.bfloat16) * 0.1).requires_grad_()
    g = torch.randn(4, 256, 640, device="cuda", dtype=torch.bfloat16)
    outs = {}
    for mode in ("lib", "vcx"):
        xi = x.clone().requires_grad_()
        with config.override(gemm_fwd=mode):
            y = ops.linear(xi, w, b)
            y.backward(g)
        outs[mode] = (y.detach().float(), xi.grad.float())
        w.grad = b.grad = None
    for a, r in zip(outs["vcx"], outs["lib"]):
        assert (a - r).abs().max().item() < 1e-2 * r.abs().max().item()
