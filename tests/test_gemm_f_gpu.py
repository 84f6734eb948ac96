"""Forward GEMM in the library's geometry (csrc/kernels/gemm_f.hip: 256 x 256 tiles, 4 waves of 128 x 128 or 8 of 128 x 64;
256 x 128 (8 waves of 64 x 64) for N = 128 and 256 x 64 (4 waves of 64 x 64) for N = 64)
against an fp32 PyTorch reference: one tile, many tiles, a 128-column last panel, the shortest K (3 slices ahead of 6), ragged M (rows past
the operand read as zeros and are never stored), strided rows, refusals, and bit-identical repeats."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("waves", [4, 8])
@pytest.mark.parametrize("M,N,K", [(256, 256, 256), (4096, 2304, 768), (8192, 768, 3072), (300, 512, 192),
                                   (1000, 256, 1024), (256 * 33, 768, 768),
                                   (700, 640, 384), (512, 128, 256), (1000, 64, 576), (300, 128, 192)])
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
    assert not C.gemm_f_supported(512, 704, 768)  # N % 128 (and not 64)
    assert not C.gemm_f_supported(512, 32, 768)
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


@pytest.mark.parametrize("waves", [4, 8])
@pytest.mark.parametrize("imgs,H,W,Cin,Cout,stride", [(2, 9, 7, 64, 128, 1), (3, 8, 8, 128, 256, 2),
                                                      (1, 7, 7, 512, 128, 1), (5, 5, 6, 64, 384, 2),
                                                      (2, 14, 14, 256, 256, 1), (3, 11, 13, 64, 64, 1),
                                                      (2, 12, 12, 64, 64, 2), (1, 9, 9, 128, 64, 1)])
def test_gemm_f_conv3x3_matches_fp32(gpu, imgs, H, W, Cin, Cout, stride, waves):
    """gemm_f's implicit-GEMM mode (the patch matrix gathered by the LDS-DMA's per-lane offsets, padding taps
    as zeros) against an fp32 convolution: borders, odd and non-square images, stride 2, a ragged last row
    tile, with and without bias."""
    import torch.nn.functional as F
    from distributedvolunteercomputing_amd.ops import native

    C = native()
    assert C.gemm_f_conv3x3_supported(imgs, H, W, Cin, Cout, stride)
    torch.manual_seed(imgs * H + Cin + stride)
    x = torch.randn(imgs, H, W, Cin, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(Cout, 3, 3, Cin, device="cuda") / (3 * Cin ** 0.5)).to(torch.bfloat16)
    bias = torch.randn(Cout, device="cuda", dtype=torch.bfloat16)
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    ref = F.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), stride=stride, padding=1)
    ref = ref.permute(0, 2, 3, 1)
    y = torch.full((imgs, Ho, Wo, Cout), float("nan"), device="cuda", dtype=torch.bfloat16)
    C.gemm_f_conv3x3(x, w, y, stride, None, waves)
    torch.cuda.synchronize()
    assert (y.float() - ref).abs().max().item() < 1e-2 * ref.abs().max().item()
    C.gemm_f_conv3x3(x, w, y, stride, bias, waves)
    torch.cuda.synchronize()
    ref = ref + bias.float()
    assert (y.float() - ref).abs().max().item() < 1e-2 * ref.abs().max().item()


def test_gemm_f_conv3x3_refusals(gpu):
    from distributedvolunteercomputing_amd.ops import native

    C = native()
    assert not C.gemm_f_conv3x3_supported(2, 8, 8, 96, 128, 1)   # Cin not a power of two
    assert not C.gemm_f_conv3x3_supported(2, 8, 8, 32, 128, 1)   # Cin < 64
    assert not C.gemm_f_conv3x3_supported(2, 8, 8, 64, 96, 1)    # Cout % 128 (and not 64)
    assert not C.gemm_f_conv3x3_supported(2, 8, 8, 64, 128, 3)   # stride
    x = torch.randn(2, 8, 8, 64, device="cuda", dtype=torch.bfloat16)
    w = torch.randn(128, 3, 3, 64, device="cuda", dtype=torch.bfloat16)
    with pytest.raises(RuntimeError):
        C.gemm_f_conv3x3(x, w, torch.empty(2, 8, 8, 128, device="cuda", dtype=torch.bfloat16), 2)  # wrong out shape


@pytest.mark.parametrize("splits", [2, 4, -1])
def test_gemm_f_split_k_matches_fp32(gpu, splits):
    """Split-K (fp32 partials per split, summed with the bias by splitk_bias_kernel): explicit and automatic
    split counts, ragged M, a 128-column last panel, strided output rows."""
    from distributedvolunteercomputing_amd.ops import native

    C = native()
    torch.manual_seed(11 + splits)
    M, N, K = 700, 640, 1536
    a = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.03
    bias = torch.randn(N, device="cuda", dtype=torch.bfloat16)
    wide = torch.full((M, N + 64), float("nan"), device="cuda", dtype=torch.bfloat16)
    c = wide[:, :N]
    C.gemm_f(a, b, c, bias, 8, splits)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().t() + bias.float()
    assert (c.float() - ref).abs().max().item() < 1e-2 * ref.abs().max().item()
    assert torch.isnan(wide[:, N:].float()).all()
    assert C.gemm_f_splits(M, N, K) > 1  # 9 tiles: split to fill the CUs
    with pytest.raises(RuntimeError):
        C.gemm_f(a, b, c, bias, 8, 5)  # 48 slices do not split into 5 even parts


def test_gemm_f_conv3x3_split_k(gpu):
    """The deep-K, few-tile convolutions of ResNet-50 stage 4 take the automatic split."""
    import torch.nn.functional as F
    from distributedvolunteercomputing_amd.ops import native

    C = native()
    torch.manual_seed(2)
    x = torch.randn(4, 7, 7, 512, device="cuda", dtype=torch.bfloat16)
    w = (torch.randn(512, 3, 3, 512, device="cuda") / 70).to(torch.bfloat16)
    y = torch.empty(4, 7, 7, 512, device="cuda", dtype=torch.bfloat16)
    assert C.gemm_f_splits(4 * 49, 512, 9 * 512) > 1
    C.gemm_f_conv3x3(x, w, y, 1)
    torch.cuda.synchronize()
    ref = F.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), padding=1).permute(0, 2, 3, 1)
    assert (y.float() - ref).abs().max().item() < 1e-2 * ref.abs().max().item()


@pytest.mark.parametrize("cin,cout", [(64, 64), (128, 256), (256, 128)])
def test_gemm_f_conv3x3_flip_taps_is_the_input_gradient(gpu, cin, cout):
    """flip_taps: gemm_f_conv3x3(dy, W^T, flip_taps=True) with the UNFLIPPED transposed weight [Cin][ky][kx][Cout]
    equals the stride-1 input gradient of the convolution (fp32 oracle: torch's convolution_backward)."""
    from distributedvolunteercomputing_amd.ops import native

    C = native()
    torch.manual_seed(cin + cout)
    imgs, H, W = 3, 9, 11
    x = torch.randn(imgs, cin, H, W, device="cuda")
    w = torch.randn(cout, cin, 3, 3, device="cuda") / (3 * cin ** 0.5)
    dy = torch.randn(imgs, cout, H, W, device="cuda")
    ref = torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                              [True, False, False])[0].permute(0, 2, 3, 1)
    dyh = dy.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    wt = w.permute(1, 2, 3, 0).contiguous().to(torch.bfloat16)  # [Cin][ky][kx][Cout], taps unflipped
    dx = torch.empty(imgs, H, W, cin, device="cuda", dtype=torch.bfloat16)
    C.gemm_f_conv3x3(dyh, wt, dx, 1, flip_taps=True)
    torch.cuda.synchronize()
    assert (dx.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()


@pytest.mark.parametrize("cin,cout,imgs,hw", [(64, 64, 3, 9), (128, 256, 3, 9), (256, 128, 3, 9), (512, 512, 4, 7)])
def test_gemm_f_conv3x3_tap_major_weight(gpu, cin, cout, imgs, hw):
    """Tap-major B ([9][Cout_call][Cin_call], a 3-D w): the input gradient from the transposed channels-last weight
    matrix (transpose_bf16 of [Cout, 9 Cin] viewed [9, Cin, Cout]) with flip_taps, and a forward convolution from
    the same layout; the 512-channel case runs split-K. fp32 oracle: torch's convolution / convolution_backward."""
    import torch.nn.functional as F

    from distributedvolunteercomputing_amd.ops import native

    C = native()
    torch.manual_seed(cin * 3 + cout)
    x = torch.randn(imgs, cin, hw, hw + 2, device="cuda")
    w = torch.randn(cout, cin, 3, 3, device="cuda") / (3 * cin ** 0.5)
    dy = torch.randn(imgs, cout, hw, hw + 2, device="cuda")
    ref = torch.ops.aten.convolution_backward(dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                                              [True, False, False])[0].permute(0, 2, 3, 1)
    wb = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = C.transpose_bf16(wb.permute(0, 2, 3, 1).reshape(cout, 9 * cin)).view(9, cin, cout)
    dx = torch.empty(imgs, hw, hw + 2, cin, device="cuda", dtype=torch.bfloat16)
    C.gemm_f_conv3x3(dy.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16), wt, dx, 1, flip_taps=True)
    torch.cuda.synchronize()
    assert (dx.float() - ref).abs().max().item() < 2e-2 * ref.abs().max().item()
    # forward from a tap-major weight: w9[t][co][ci] = w[co][ci][t]
    w9 = w.permute(2, 3, 0, 1).reshape(9, cout, cin).contiguous().to(torch.bfloat16)
    y = torch.empty(imgs, hw, hw + 2, cout, device="cuda", dtype=torch.bfloat16)
    C.gemm_f_conv3x3(x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16), w9, y, 1)
    torch.cuda.synchronize()
    yref = F.conv2d(x, w, padding=1).permute(0, 2, 3, 1)
    assert (y.float() - yref).abs().max().item() < 2e-2 * yref.abs().max().item()
