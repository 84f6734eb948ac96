"""3x3 convolution weight gradient on the hand-written gemm_wg with the patch matrix of x gathered while
staging (csrc/kernels/gemm_wg.hip IMPL, bindings gemm_wg_conv3x3; models/resnet.py Conv3x3): against the fp32
torch weight gradient of the same bf16 operands, at the ResNet-50 stage-2/3/4 channel counts, stride 1 and 2,
including the zero padding at every image border and accumulation into an existing gradient."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def C(gpu):
    from distributedvolunteercomputing_amd.ops._lib import native

    return native()


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm())


# (imgs, H, Cin, Cout, stride): tokens = imgs * Ho * Wo is a multiple of 64
SHAPES = [(16, 14, 256, 256, 1), (64, 7, 512, 512, 1), (16, 28, 256, 256, 2), (16, 14, 256, 512, 1),
          (64, 14, 512, 256, 2), (4, 32, 256, 256, 1),
          # 128 channels (ResNet-50 stage 2): 2 taps per 256-column block, ragged last block (1152 columns),
          # ragged output rows (Cout = 128 of a 256-row tile)
          (16, 28, 128, 128, 1), (16, 56, 128, 128, 2), (8, 28, 128, 256, 1), (8, 28, 256, 128, 1)]


@pytest.mark.parametrize("imgs,H,cin,cout,s", SHAPES)
def test_conv3x3_wgrad_matches_fp32(C, gpu, imgs, H, cin, cout, s):
    torch.manual_seed(imgs + H + cin + s)
    x = torch.randn(imgs, H, H, cin, device=gpu).to(torch.bfloat16)  # NHWC
    Ho = (H - 1) // s + 1
    dy = torch.randn(imgs, Ho, Ho, cout, device=gpu).to(torch.bfloat16)
    assert C.gemm_wg_conv3x3_supported(cout, cin, imgs, H, H, s)
    ref = torch.nn.grad.conv2d_weight(x.permute(0, 3, 1, 2).float(), (cout, cin, 3, 3), dy.permute(0, 3, 1, 2).float(),
                                      stride=s, padding=1)  # [Cout, Cin, 3, 3]
    ref_cl = ref.permute(0, 2, 3, 1).reshape(cout, 9 * cin)  # [Cout][ky][kx][Cin]
    out = torch.empty(cout, 9 * cin, device=gpu, dtype=torch.bfloat16)
    C.gemm_wg_conv3x3(dy, x, out, False, s)
    assert _rel(out, ref_cl) < 1e-2
    base = torch.randn(cout, 9 * cin, device=gpu).to(torch.bfloat16)
    acc = base.clone()
    C.gemm_wg_conv3x3(dy, x, acc, True, s)
    assert _rel(acc, base.float() + ref_cl) < 1e-2


def test_conv3x3_wgrad_refuses_untiled_shapes(C):
    assert not C.gemm_wg_conv3x3_supported(64, 64, 128, 56, 56, 1)    # Cout, Cin % 128
    assert not C.gemm_wg_conv3x3_supported(256, 256, 3, 14, 14, 1)    # 588 tokens: not a multiple of 64
    assert not C.gemm_wg_conv3x3_supported(256, 256, 16, 14, 14, 3)   # stride


@pytest.mark.parametrize("preset_grad", [False, True])
def test_resnet_conv3x3_module_grads(gpu, preset_grad):
    """models/resnet.Conv3x3 on the gemm_wg path: input and weight gradients against the fp32 reference, with
    the weight gradient returned to autograd or accumulated straight into a preset channels-last .grad (the
    flat gradient buffer's case)."""
    from distributedvolunteercomputing_amd.models.resnet import Conv3x3

    torch.manual_seed(3)
    m = Conv3x3(256, 256, stride=2).to(gpu, torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(16, 256, 28, 28, device=gpu).to(torch.bfloat16).to(memory_format=torch.channels_last)
    x.requires_grad_()
    assert m.vcx_wgrad(x)
    r = torch.randn(16, 256, 14, 14, device=gpu)
    g0 = None
    if preset_grad:
        g0 = torch.randn_like(m.weight).to(memory_format=torch.channels_last)
        m.weight.grad = g0.clone()
    (m(x).float() * r).sum().backward()
    xr = x.detach().float().requires_grad_()
    wr = m.weight.detach().float().requires_grad_()
    (F.conv2d(xr, wr, None, 2, 1) * r).sum().backward()
    want_w = wr.grad + (g0.float() if preset_grad else 0)
    assert _rel(m.weight.grad, want_w) < 1e-2
    assert _rel(x.grad, xr.grad) < 1e-2


@pytest.mark.parametrize("fwd,wgrad,stride,ch", [("vcx", "vcx", 1, 256), ("vcx", "lib", 1, 256), ("lib", "vcx", 1, 256),
                                                 ("vcx", "vcx", 2, 256), ("vcx", "lib", 2, 256), ("vcx", "vcx", 1, 128),
                                                 ("vcx", "vcx", 2, 128), ("vcx", "vcx", 1, 64)])
def test_resnet_conv3x3_module_on_gemm_f(gpu, fwd, wgrad, stride, ch):
    """models/resnet.Conv3x3 with the forward (and, at stride 1, the input gradient) on gemm_f's implicit GEMM
    in every combination with the weight-gradient path: output, input and weight gradients against fp32; the
    128- and 64-channel stages on its 256 x 128 / 256 x 64 tiles (weight gradient on MIOpen there)."""
    from distributedvolunteercomputing_amd import config
    from distributedvolunteercomputing_amd.models.resnet import Conv3x3

    torch.manual_seed(5 + stride)
    m = Conv3x3(ch, ch, stride=stride).to(gpu, torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(8, ch, 14, 14, device=gpu).to(torch.bfloat16).to(memory_format=torch.channels_last)
    x.requires_grad_()
    Ho = (14 - 1) // stride + 1
    r = torch.randn(8, ch, Ho, Ho, device=gpu)
    with config.override(conv3x3_fwd=fwd, conv3x3_wgrad=wgrad):
        from distributedvolunteercomputing_amd.models import resnet

        assert resnet._fwd_vcx(8, 14, 14, ch, ch, stride) == (fwd == "vcx")  # the path under test is taken
        y = m(x)
        (y.float() * r).sum().backward()
    xr = x.detach().float().requires_grad_()
    wr = m.weight.detach().float().requires_grad_()
    yr = F.conv2d(xr, wr, None, stride, 1)
    (yr * r).sum().backward()
    assert _rel(y, yr) < 1e-2
    assert _rel(m.weight.grad, wr.grad) < 1e-2
    assert _rel(x.grad, xr.grad) < 1e-2
