"""Hand-written weight-gradient GEMM (csrc/kernels/gemm.hip gemm_tn: token-major operands read
transposed out of LDS by ds_read_b64_tr_b16, split-K fp32 partials) against an fp32 torch oracle."""
import pytest
import torch

from distributedvolunteercomputing_amd import config

pytestmark = pytest.mark.gpu


def _ref(dy, x):
    return dy.float().t() @ x.float()


@pytest.mark.parametrize("M,N,K,splits", [(4096, 768, 3072, 7), (4096, 3072, 768, 7), (8192, 2304, 768, 9),
                                          (2048, 768, 768, 10), (1024, 256, 512, 1), (8192, 512, 256, 3)])
def test_gemm_tn_matches_fp32(gpu, M, N, K, splits):
    from distributedvolunteercomputing_amd.ops import native

    g = torch.Generator(device=gpu).manual_seed(M + N + K)
    dy = torch.randn(M, N, device=gpu, generator=g).to(torch.bfloat16)
    x = torch.randn(M, K, device=gpu, generator=g).to(torch.bfloat16)
    out = torch.empty(N, K, device=gpu, dtype=torch.bfloat16)
    native().gemm_tn(dy, x, out, splits, False)
    ref = _ref(dy, x)
    err = (out.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 8e-3 * scale, (err, scale)
    # accumulate into an existing gradient
    base = torch.randn(N, K, device=gpu, generator=g).to(torch.bfloat16)
    acc = base.clone()
    native().gemm_tn(dy, x, acc, splits, True)
    err2 = (acc.float() - (ref + base.float())).abs().max().item()
    assert err2 <= 8e-3 * scale, (err2, scale)


def test_gemm_tn_strided_rows_and_wgrad_route(gpu):
    """Operands that are column slices of wider rows (lda > M), and the Linear wgrad path with
    VCX_GEMM_WGRAD=vcx producing the same gradient as the library path."""
    import importlib

    from distributedvolunteercomputing_amd.ops import native

    linear = importlib.import_module("distributedvolunteercomputing_amd.ops.linear")

    g = torch.Generator(device=gpu).manual_seed(7)
    big = torch.randn(4096, 1024, device=gpu, generator=g).to(torch.bfloat16)
    dy = big[:, :768]
    x = torch.randn(4096, 512, device=gpu, generator=g).to(torch.bfloat16)
    out = torch.empty(768, 512, device=gpu, dtype=torch.bfloat16)
    native().gemm_tn(dy, x, out, 4, False)
    ref = _ref(dy, x)
    assert (out.float() - ref).abs().max().item() <= 8e-3 * ref.abs().max().item()
    with config.override(gemm_wgrad="vcx"):
        assert linear.gemm_tn_ok(4096, 768, 512, dy)
        gv = linear.wgrad(dy.contiguous(), x)
    with config.override(gemm_wgrad="lib"):
        gl = linear.wgrad(dy.contiguous(), x)
    assert (gv.float() - gl.float()).abs().max().item() <= 1e-2 * ref.abs().max().item()
