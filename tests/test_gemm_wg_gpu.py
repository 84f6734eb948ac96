"""Weight-gradient GEMM gemm_wg (csrc/kernels/gemm_wg.hip: LDS ring staged by inline-asm LDS-DMA,
token-major operands read transposed by ds_read_b64_tr_b16, split-K fp32 partials) against an fp32
torch oracle, for both loader geometries (all 8 waves stage, or waves 0-3 only), with ragged splits,
strided rows, accumulation into a gradient, and the Linear backward routing to it by default."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(dy, x):
    return dy.float().t() @ x.float()


@pytest.mark.parametrize("M,N,K,splits", [(4096, 768, 3072, 7), (4096, 3072, 768, 7), (8192, 2304, 768, 9),
                                          (2048, 768, 768, 10), (1024, 256, 512, 1), (8192, 512, 256, 3),
                                          (65536, 768, 768, 28), (4096, 1152, 768, 3), (8192, 640, 512, 2)])
def test_gemm_wg_matches_fp32(gpu, M, N, K, splits):
    from distributedvolunteercomputing_amd.ops import native

    C = native()
    g = torch.Generator(device=gpu).manual_seed(M + N + K)
    dy = torch.randn(M, N, device=gpu, generator=g).to(torch.bfloat16)
    x = torch.randn(M, K, device=gpu, generator=g).to(torch.bfloat16)
    ref = _ref(dy, x)
    scale = ref.abs().max().item()
    for loaders in (8, 4):
        out = torch.full((N, K), float("nan"), device=gpu, dtype=torch.bfloat16)
        C.gemm_wg(dy, x, out, False, splits, loaders)
        err = (out.float() - ref).abs().max().item()
        assert err <= 8e-3 * scale, (loaders, err, scale)
    # accumulate into an existing gradient (the flat .grad path)
    base = torch.randn(N, K, device=gpu, generator=g).to(torch.bfloat16)
    acc = base.clone()
    C.gemm_wg(dy, x, acc, True, splits)
    err2 = (acc.float() - (ref + base.float())).abs().max().item()
    assert err2 <= 8e-3 * scale, (err2, scale)


def test_gemm_wg_strided_rows_default_splits_and_refusals(gpu):
    from distributedvolunteercomputing_amd.ops import native

    C = native()
    g = torch.Generator(device=gpu).manual_seed(7)
    big = torch.randn(4096, 1024, device=gpu, generator=g).to(torch.bfloat16)
    dy = big[:, :768]  # lda = 1024
    x = torch.randn(4096, 512, device=gpu, generator=g).to(torch.bfloat16)
    out = torch.empty(768, 512, device=gpu, dtype=torch.bfloat16)
    C.gemm_wg(dy, x, out)  # default splits and prefetch distance
    ref = _ref(dy, x)
    assert (out.float() - ref).abs().max().item() <= 8e-3 * ref.abs().max().item()
    assert not C.gemm_wg_supported(768, 500, 4096)  # N % 256
    assert not C.gemm_wg_supported(768, 512, 4000)  # tokens % 64
    with pytest.raises(RuntimeError):
        C.gemm_wg(dy, x, out, False, 0, 5)  # no such loader geometry
    # the Linear backward takes gemm_wg by default and agrees with the library path
    import importlib

    from distributedvolunteercomputing_amd import config

    linear = importlib.import_module("distributedvolunteercomputing_amd.ops.linear")
    dyc = dy.contiguous()
    assert linear.gemm_wg_ok(4096, 768, 512, dyc)
    gv = linear.wgrad(dyc, x)
    with config.override(gemm_wgrad="lib"):
        assert not linear.gemm_wg_ok(4096, 768, 512, dyc)
        gl = linear.wgrad(dyc, x)
    assert (gv.float() - gl.float()).abs().max().item() <= 1e-2 * ref.abs().max().item()


def test_gemm_wg_repeat_runs_bit_identical(gpu):
    """No atomics anywhere: repeats must match bit for bit (a slot read before its LDS-DMA landed
    would show as differing tiles from run to run)."""
    from distributedvolunteercomputing_amd.ops import native

    C = native()
    g = torch.Generator(device=gpu).manual_seed(11)
    dy = torch.randn(16384, 2304, device=gpu, generator=g).to(torch.bfloat16)
    x = torch.randn(16384, 768, device=gpu, generator=g).to(torch.bfloat16)
    out = torch.empty(2304, 768, device=gpu, dtype=torch.bfloat16)
    C.gemm_wg(dy, x, out)
    first = out.clone()
    for _ in range(10):
        C.gemm_wg(dy, x, out)
        assert torch.equal(out, first)


def test_gemm_wg_lm_head_shape_default_splits(gpu):
    """The GPT-2 LM head's weight gradient [50304, 768] over 65536 tokens (ops/linear.py gemm_wg_ok,
    config.wgrad_wide): 591 tiles with a ragged last row panel (50304 = 196.5 x 256) whose lanes past the
    last column re-read valid data (the logit gradient ends at its allocation's end), the default 4 token
    splits (each split's [16384, 50304] panel 1.65 GB, under the 2 GB offset limit)."""
    from distributedvolunteercomputing_amd.ops import native
    from distributedvolunteercomputing_amd.ops.linear import gemm_wg_ok

    C = native()
    T, V, D = 65536, 50304, 768
    assert C.gemm_wg_supported(V, D, T) and gemm_wg_ok(T, V, D, torch.empty(1, device=gpu, dtype=torch.bfloat16))
    g = torch.Generator(device=gpu).manual_seed(11)
    dy = (torch.randn(T, V, device=gpu, generator=g, dtype=torch.bfloat16) * 0.01)
    x = torch.randn(T, D, device=gpu, generator=g).to(torch.bfloat16)
    ref = torch.zeros(V, D, device=gpu)
    for i in range(0, T, 8192):
        ref += dy[i:i + 8192].float().t() @ x[i:i + 8192].float()
    out = torch.full((V, D), float("nan"), device=gpu, dtype=torch.bfloat16)
    C.gemm_wg(dy, x, out)
    scale = ref.abs().max().item()
    assert torch.isfinite(out.float()).all()
    err = (out.float() - ref).abs().max().item()
    assert err <= 8e-3 * scale, (err, scale)

