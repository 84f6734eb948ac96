"""Llama-3 and ResNet models on the GPU (HIP RMSNorm/SwiGLU/xent paths vs reference ops)."""
import pytest
import torch

from distributedvolunteercomputing_amd.models.llama import Llama, LlamaConfig
from distributedvolunteercomputing_amd.models.resnet import resnet_tiny
from distributedvolunteercomputing_amd.ops._lib import reference_ops
from distributedvolunteercomputing_amd.parallel.compression import PowerSGDCompressor
from distributedvolunteercomputing_amd.parallel.zero import ShardedConfig, ShardedDPTrainer

pytestmark = pytest.mark.gpu


def test_llama_tiny_matches_reference(gpu):
    cfg = LlamaConfig.preset("llama-tiny")
    m = Llama(cfg).to(gpu, torch.bfloat16)
    x = torch.randint(0, cfg.vocab_size, (2, 64), device=gpu)
    loss = m(x, x.roll(-1, 1))
    loss.backward()
    g1 = {n: p.grad.float().clone() for n, p in m.named_parameters()}
    m.zero_grad(set_to_none=True)
    with reference_ops():
        lr = m(x, x.roll(-1, 1))
        lr.backward()
    assert abs(loss.item() - lr.item()) < 2e-2
    for n, p in m.named_parameters():
        rel = (g1[n] - p.grad.float()).norm() / (p.grad.float().norm() + 1e-6)
        assert rel < 0.08, (n, float(rel))


def _oracle_compare(m, loss_fn, tol, slack=1.25, chaotic=1.0):
    """Run `loss_fn` on the bf16 model through the HIP path, then (reference ops) on the same bf16
    model and on an fp32 copy (the oracle); every parameter gradient of the HIP path must be
    within `tol` of the oracle and no worse than the torch bf16 path's own error (+25 %)."""
    import copy

    oracle = copy.deepcopy(m).float()
    loss = loss_fn(m)
    loss.backward()
    g_native = {n: p.grad.float().clone() for n, p in m.named_parameters()}
    m.zero_grad(set_to_none=True)
    with reference_ops():
        lb = loss_fn(m)
        lb.backward()
        lo = loss_fn(oracle)
        lo.backward()
    g_bf16 = {n: p.grad.float() for n, p in m.named_parameters()}
    assert abs(loss.item() - lo.item()) < 1e-2 * abs(lo.item()) + 1e-3, (loss.item(), lo.item())
    errs = {}
    for n, po in oracle.named_parameters():
        ref = po.grad.float()
        den = ref.norm().item()
        if den == 0:
            continue
        e_nat = (g_native[n] - ref).norm().item() / den
        e_t = (g_bf16[n] - ref).norm().item() / den
        errs[n] = (round(e_nat, 4), round(e_t, 4))
        # the absolute bound applies where bf16 arithmetic itself can meet it: a gradient that the
        # plain torch bf16 path already misses by more (e.g. a ResNet stem weight summed over every
        # pixel through train-mode BatchNorm, measured 0.37 on both paths) is held to that path.
        # Where the torch bf16 path is off by more than `chaotic` (10-60 % on a few train-mode BN
        # parameters of the tiny ResNet: rounding differences amplified through the batch
        # statistics), the two bf16 paths round differently and land anywhere in that error
        # ball: there the HIP path must stay within 1.6x of torch's error (scripts/bn_diag.py:
        # the fused BN kernels are themselves MORE accurate than torch's bf16 BN on every tensor)
        bound = (1.6 if e_t > chaotic else slack) * e_t + 2e-3
        assert e_nat < max(tol, bound), (n, e_nat, e_t)
        assert e_nat <= bound, (n, e_nat, e_t)
    return errs


def test_llama_tiny_gradients_vs_fp32_oracle(gpu):
    """Llama-tiny (HIP RMSNorm, RoPE+QKV split, GQA flash attention, SwiGLU, fused xent) against an
    fp32 copy of itself through the plain torch ops, every parameter gradient."""
    torch.manual_seed(5)
    cfg = LlamaConfig.preset("llama-tiny")
    m = Llama(cfg).to(gpu, torch.bfloat16)
    x = torch.randint(0, cfg.vocab_size, (2, 128), device=gpu)
    errs = _oracle_compare(m, lambda mm: mm(x, x.roll(-1, 1)), tol=0.03)
    assert len(errs) == len(list(m.parameters()))


def test_resnet_bottlenecks_vs_fp32_oracle(gpu):
    """A ResNet bottleneck stack (bf16, channels-last MIOpen convolutions, train-mode BatchNorm)
    against its fp32 copy: loss and every parameter gradient (the zero-initialised last BN of each
    residual branch gets random weights so the branch gradients are not trivially zero)."""
    torch.manual_seed(6)
    m = resnet_tiny().to(gpu)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            torch.nn.init.uniform_(mod.weight, 0.5, 1.5)
            torch.nn.init.uniform_(mod.bias, -0.1, 0.1)
    m = m.to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(16, 3, 32, 32, device=gpu)
    y = torch.randint(0, 10, (16,), device=gpu)

    def loss_fn(mm):
        dt = next(mm.parameters()).dtype
        return mm(x.to(dt).to(memory_format=torch.channels_last), y)

    _oracle_compare(m, loss_fn, tol=0.06, chaotic=0.1)


def test_resnet_identity_shortcut_gradient_join(gpu):
    """Identity-shortcut bottlenecks (ResNet with 2 blocks per stage) take the shortcut's gradient into
    conv1's input-gradient GEMM (ops/linear.py GradJoin, beta = 1: one rounding) instead of autograd's
    bf16 add; projection-shortcut blocks (stride 1 and 2) add the shortcut convolution's input gradient
    into the one conv1 deposited. Against an fp32 oracle of the same model, the joined gradients (input
    and every parameter) are no worse than the unjoined ones."""
    import copy

    from distributedvolunteercomputing_amd.models import resnet as R

    torch.manual_seed(8)
    m = R.ResNet((2, 2), n_classes=10, width=16).to(gpu)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            torch.nn.init.uniform_(mod.weight, 0.5, 1.5)
    oracle = copy.deepcopy(m)
    m = m.to(torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(16, 3, 32, 32, device=gpu)
    y = torch.randint(0, 10, (16,), device=gpu)
    probe = lambda c: torch.empty(1, c, 4, 4, device=gpu, dtype=torch.bfloat16).to(memory_format=torch.channels_last)  # noqa: E731
    assert sorted(b.down[0].stride[0] for b in m.blocks if b.down is not None) == [1, 2]
    assert all(b.conv1.gemm_path(probe(b.conv1.in_channels)) for b in m.blocks)
    assert all(b.down[0].gemm_path(probe(b.conv1.in_channels)) for b in m.blocks if b.down is not None)

    def grads(model, join_on, dt):
        orig = R.GradJoin
        if not join_on:
            R.GradJoin = lambda: None  # noqa: E731 -- every block falls back to autograd's add
        try:
            xi = x.to(dt).to(memory_format=torch.channels_last).requires_grad_()
            model.zero_grad(set_to_none=True)
            model(xi, y).backward()
            return [xi.grad.float()] + [p.grad.float() for p in model.parameters()]
        finally:
            R.GradJoin = orig

    takes, orig_take = [], R.GradJoin.take

    def take(self):
        g = orig_take(self)
        takes.append(g is not None)
        return g

    R.GradJoin.take = take
    try:
        gj = grads(m, True, torch.bfloat16)
    finally:
        R.GradJoin.take = orig_take
    assert takes.count(True) == len(m.blocks), takes  # every block's second side found the first's gradient
    gn = grads(m, False, torch.bfloat16)
    with reference_ops():
        go = grads(oracle, True, torch.float32)
    for i, (a_, b_, o_) in enumerate(zip(gj, gn, go)):
        den = o_.norm().item()
        if den == 0:
            continue
        ej, en = (a_ - o_).norm().item() / den, (b_ - o_).norm().item() / den
        assert ej <= 1.25 * en + 1e-2, (i, ej, en)


def test_llama_sharded_powersgd_trains(gpu):
    cfg = LlamaConfig.preset("llama-tiny")
    m = Llama(cfg).to(gpu, torch.bfloat16)
    tr = ShardedDPTrainer(m, ShardedConfig(lr=3e-3, weight_decay=0.0), device=gpu)
    tr.compressor = PowerSGDCompressor(tr.flat, rank=4, device=gpu)
    x = torch.randint(0, cfg.vocab_size, (4, 64), device=gpu)
    losses = [float(tr.step(x, x.roll(-1, 1))) for _ in range(25)]
    assert losses[-1] < losses[0] - 0.5, losses


def test_resnet_tiny_local_sgd_topk_trains(gpu):
    from distributedvolunteercomputing_amd.parallel.compression import TopKCompressor
    from distributedvolunteercomputing_amd.parallel.local_sgd import LocalSGDConfig, LocalSGDTrainer

    m = resnet_tiny().to(gpu, torch.bfloat16).to(memory_format=torch.channels_last)
    tr = LocalSGDTrainer(m, LocalSGDConfig(H=2, lr=1e-3), device=gpu)
    tr.compressor = TopKCompressor(tr.flat.numel, 0.05, gpu)
    x = torch.randn(8, 3, 32, 32, device=gpu).to(torch.bfloat16).to(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=gpu)
    losses = []
    for _ in range(12):
        st = tr.step(x, y)
        losses.append(float(st.extra["loss_t"]))
    torch.cuda.synchronize()
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < losses[0], losses  # top-k + error feedback still fits one batch


def test_rope_qkv_matches_reference(gpu):
    """HIP rotary embedding fused with the QKV split vs the torch reference (fwd + bwd)."""
    from distributedvolunteercomputing_amd import ops
    from distributedvolunteercomputing_amd.ops.rope import apply_rope, rope_tables

    torch.manual_seed(0)
    B, T, Hq, Hkv, hd = 2, 100, 8, 2, 128
    qkv = torch.randn(B, T, (Hq + 2 * Hkv) * hd, device=gpu).to(torch.bfloat16).requires_grad_()
    cos, sin = rope_tables(T, hd, 500000.0, gpu)
    q, k, v = ops.rope_qkv(qkv, cos, sin, Hq, Hkv)
    x32 = qkv.detach().float().requires_grad_()
    qr, kr, vr = x32.split([Hq * hd, Hkv * hd, Hkv * hd], -1)
    qr = apply_rope(qr.reshape(B, T, Hq, hd).transpose(1, 2), cos, sin)
    kr = apply_rope(kr.reshape(B, T, Hkv, hd).transpose(1, 2), cos, sin)
    vr = vr.reshape(B, T, Hkv, hd).transpose(1, 2)
    for a, r in ((q, qr), (k, kr), (v, vr)):
        assert a.shape == r.shape
        assert torch.allclose(a.float(), r, atol=3e-2, rtol=2e-2)
    gs = [torch.randn_like(r) for r in (qr, kr, vr)]
    sum((a.float() * g).sum() for a, g in zip((q, k, v), gs)).backward()
    sum((r * g).sum() for r, g in zip((qr, kr, vr), gs)).backward()
    rel = float((qkv.grad.float() - x32.grad).norm() / x32.grad.norm())
    assert rel < 1e-2, rel


@pytest.mark.parametrize("stride,cin,cout,narrow", [(1, 64, 256, "lib"), (2, 64, 256, "lib"), (1, 256, 64, "vision"),
                                                    (1, 64, 64, "vision"), (2, 128, 64, "vision")])
def test_resnet_conv1x1_gemm_matches_conv(gpu, stride, cin, cout, narrow):
    """The ResNet 1x1 convolution as a GEMM on the NHWC view (models/resnet.py Conv1x1) against an
    fp32 F.conv2d: output, input gradient and weight gradient, stride 1 and 2; narrow outputs (<= 128
    channels) also on the vision GEMM (config.narrow_gemm)."""
    from distributedvolunteercomputing_amd import config
    from distributedvolunteercomputing_amd.models.resnet import Conv1x1

    with config.override(narrow_gemm=narrow):
        _conv1x1_vs_conv(gpu, stride, cin, cout)


def _conv1x1_vs_conv(gpu, stride, cin, cout):
    torch.manual_seed(stride)
    from distributedvolunteercomputing_amd.models.resnet import Conv1x1

    conv = Conv1x1(cin, cout, stride=stride).to(gpu, torch.bfloat16)
    x = torch.randn(48, cin, 56, 56, device=gpu).to(torch.bfloat16).to(memory_format=torch.channels_last)
    x.requires_grad_()
    y = conv(x)
    assert y.is_contiguous(memory_format=torch.channels_last)
    g = torch.randn_like(y.float())
    y.backward(g.to(y.dtype))
    x32 = x.detach().float().requires_grad_()
    w32 = conv.weight.detach().float().requires_grad_()
    y32 = torch.nn.functional.conv2d(x32, w32, stride=stride)
    y32.backward(g)
    for a, r in ((y.float(), y32), (x.grad.float(), x32.grad), (conv.weight.grad.float(), w32.grad)):
        assert (a - r).norm() / r.norm() < 1e-2, float((a - r).norm() / r.norm())
    # a preset contiguous .grad of the [Cout, Cin, 1, 1] parameter (the trainer's flat-buffer view) is
    # accumulated into in place by the weight-gradient GEMM
    pre = torch.randn_like(conv.weight)
    conv.weight.grad = pre.clone()
    buf = conv.weight.grad
    conv(x).backward(g.to(y.dtype))
    assert conv.weight.grad.data_ptr() == buf.data_ptr()
    ref = pre.float() + w32.grad
    assert (conv.weight.grad.float() - ref).norm() / ref.norm() < 1e-2


@pytest.mark.parametrize("C,res,relu", [(64, False, True), (256, True, True), (2048, True, True), (512, False, False)])
def test_fused_batchnorm_act_vs_fp32(gpu, C, res, relu):
    """Train-mode BatchNorm (+ residual) (+ ReLU) on channels-last bf16 (csrc/kernels/batchnorm.hip)
    against torch in fp32: output, input / residual / gamma / beta gradients, running statistics."""
    from distributedvolunteercomputing_amd.ops.batchnorm import bn_act

    torch.manual_seed(C)
    bn = torch.nn.BatchNorm2d(C).to(gpu)
    torch.nn.init.uniform_(bn.weight, 0.5, 1.5)
    torch.nn.init.uniform_(bn.bias, -0.5, 0.5)
    bn32 = torch.nn.BatchNorm2d(C).to(gpu)
    bn32.load_state_dict(bn.state_dict())
    bn = bn.to(torch.bfloat16)
    H = 7 if C >= 1024 else 14
    x = (torch.randn(16, C, H, H, device=gpu) * 2 + 0.5).to(torch.bfloat16).to(memory_format=torch.channels_last)
    r = torch.randn_like(x) if res else None
    x.requires_grad_()
    if r is not None:
        r.requires_grad_()
    y = bn_act(x, bn, r, relu)
    assert type(y.grad_fn).__name__ == "_BNActBackward"  # the HIP kernels ran, not the torch fallback
    g = torch.randn_like(y)
    y.backward(g)
    x32 = x.detach().float().requires_grad_()
    r32 = r.detach().float().requires_grad_() if res else None
    y32 = bn32(x32)
    if res:
        y32 = y32 + r32
    if relu:
        y32 = torch.relu(y32)
    y32.backward(g.float())
    # torch's own bf16 BatchNorm (+ add + ReLU) on the same inputs: the accuracy bf16 storage allows
    # (dx / dres / dgamma / dbeta of a ReLU output: elements near 0 round to the other side of the
    # mask; measured 0.018-0.033 for torch, 0.018-0.024 for the fused kernels, scripts/bn_diag.py)
    bnt = torch.nn.BatchNorm2d(C).to(gpu)
    bnt.load_state_dict(bn32.state_dict())
    bnt = bnt.to(torch.bfloat16)
    xt = x.detach().clone().requires_grad_()
    rt = r.detach().clone().requires_grad_() if res else None
    with reference_ops():
        yt = bnt(xt)
        if res:
            yt = yt + rt
        if relu:
            yt = torch.relu(yt)
        yt.backward(g)
    rel = lambda a, b: float((a.float() - b).norm() / (b.norm() + 1e-6))  # noqa: E731

    def ok(a, t, ref, tol):
        e, et = rel(a, ref), rel(t, ref)
        assert e < max(tol, 1.1 * et), (e, et)

    ok(y, yt, y32, 1e-2)
    ok(x.grad, xt.grad, x32.grad, 1e-2)
    if res:
        ok(r.grad, rt.grad, r32.grad, 1e-2)
    ok(bn.weight.grad, bnt.weight.grad, bn32.weight.grad, 1e-2)
    ok(bn.bias.grad, bnt.bias.grad, bn32.bias.grad, 1e-2)
    assert rel(bn.running_mean, bn32.running_mean) < 2e-2 and rel(bn.running_var, bn32.running_var) < 2e-2
    # counted on the device by the statistics kernel's last block
    assert int(bn.num_batches_tracked) == int(bn32.num_batches_tracked) == 1
    # the shared workspace was left zeroed: a second pass gives the same output and gradients (up to
    # the order of the fp32 atomic sums; a workspace left holding the first pass's sums would double them)
    x.grad = None
    gw1, gb1 = bn.weight.grad.float(), bn.bias.grad.float()
    bn.weight.grad = bn.bias.grad = None
    y2 = bn_act(x, bn, r, relu)
    y2.backward(g)
    assert rel(y2, y.float()) < 1e-3 and rel(bn.weight.grad, gw1) < 1e-3 and rel(bn.bias.grad, gb1) < 1e-3
    assert int(bn.num_batches_tracked) == 2


def test_fused_batchnorm_layer_workspace_out_of_order_calls(gpu):
    """The per-layer workspace (finalize inside the apply / dx passes, ops/batchnorm.py _LayerWS) against the
    shared-workspace path (separate finalize kernels, self-contained per call) for call orders that break
    the steady state: a no-grad train-mode forward, two forwards before their backwards (in reverse
    order), and a second backward through a retained graph. Outputs, gradients and running stats match."""
    from distributedvolunteercomputing_amd import config
    from distributedvolunteercomputing_amd.ops.batchnorm import bn_act

    torch.manual_seed(5)
    C = 128
    xs = [(torch.randn(8, C, 14, 14, device=gpu) * (1 + i) + i).to(torch.bfloat16).to(memory_format=torch.channels_last)
          for i in range(3)]
    gs = [torch.randn_like(x) for x in xs]

    def run(layer_ws):
        torch.manual_seed(6)  # the same gamma in both runs
        bn = torch.nn.BatchNorm2d(C).to(gpu)
        torch.nn.init.uniform_(bn.weight, 0.5, 1.5)
        bn = bn.to(torch.bfloat16)
        outs, grads = [], []
        with config.override(bn_layer_ws=layer_ws):
            with torch.no_grad():
                outs.append(bn_act(xs[0], bn, None, True))  # forward without a backward
            a = xs[1].clone().requires_grad_()
            b = xs[2].clone().requires_grad_()
            ya = bn_act(a, bn, None, True)
            yb = bn_act(b, bn, None, True)  # two forwards pending
            assert type(yb.grad_fn).__name__ == "_BNActBackward"
            yb.backward(gs[2], retain_graph=True)
            ya.backward(gs[1])
            grads += [a.grad.clone(), b.grad.clone(), bn.weight.grad.clone(), bn.bias.grad.clone()]
            b.grad = None
            yb.backward(gs[2])  # second backward through the retained graph
            grads.append(b.grad.clone())
            ya2 = bn_act(a, bn, None, True)  # back in steady state
            a.grad = None
            ya2.backward(gs[1])
            grads.append(a.grad.clone())
            outs += [ya, yb, ya2]
        return outs, grads, (bn.running_mean.float(), bn.running_var.float())

    o1, g1, r1 = run(True)
    o0, g0, r0 = run(False)
    rel = lambda a, b: float((a.float() - b.float()).norm() / (b.float().norm() + 1e-6))  # noqa: E731
    for a, b in zip(o1 + g1 + list(r1), o0 + g0 + list(r0)):
        assert rel(a, b) < 2e-3, rel(a, b)


@pytest.mark.parametrize("C", [64, 1024])
def test_fused_batchnorm_grads_into_flat_buffers(gpu, C):
    """With preset contiguous .grad buffers (the trainer's flat gradient views) the BN backward ADDS
    dgamma / dbeta into them in its reduction kernel and hands autograd None; the result equals the
    returned-gradient path plus the preset values. Only one parameter needing a gradient falls back."""
    from distributedvolunteercomputing_amd.ops.batchnorm import bn_act

    torch.manual_seed(C + 1)
    bn = torch.nn.BatchNorm2d(C).to(gpu)
    torch.nn.init.uniform_(bn.weight, 0.5, 1.5)
    torch.nn.init.uniform_(bn.bias, -0.5, 0.5)
    bn = bn.to(torch.bfloat16)
    x = (torch.randn(8, C, 14, 14, device=gpu)).to(torch.bfloat16).to(memory_format=torch.channels_last)
    g = torch.randn_like(x)
    bn_act(x, bn, None, True).backward(g)  # returned-gradient path (no preset .grad)
    ref_w, ref_b = bn.weight.grad.float(), bn.bias.grad.float()
    pw = torch.randn(C, device=gpu).to(torch.bfloat16)
    pb = torch.randn(C, device=gpu).to(torch.bfloat16)
    bn.weight.grad, bn.bias.grad = pw.clone(), pb.clone()
    bn_act(x, bn, None, True).backward(g)
    rel = lambda a, b: float((a.float() - b).norm() / (b.norm() + 1e-6))  # noqa: E731
    assert rel(bn.weight.grad, pw.float() + ref_w) < 1e-2
    assert rel(bn.bias.grad, pb.float() + ref_b) < 1e-2
    bn.bias.requires_grad_(False)
    bn.weight.grad = None
    bn_act(x, bn, None, True).backward(g)
    assert rel(bn.weight.grad, ref_w) < 1e-2


@pytest.mark.parametrize("shape,ties", [((8, 64, 112, 112), False), ((3, 16, 15, 17), False), ((4, 8, 9, 10), True)])
def test_stem_maxpool_matches_torch(gpu, shape, ties):
    """The ResNet stem max-pool (3x3 / 2 / pad 1, channels-last bf16, ops/batchnorm.py stem_maxpool) against
    torch's max_pool2d on the same bf16 input: identical output, and the same input gradient (ties: the
    first maximum of the window in scan order takes the gradient, as in torch)."""
    from distributedvolunteercomputing_amd.ops.batchnorm import stem_maxpool

    torch.manual_seed(sum(shape))
    if ties:
        x = torch.randint(-2, 3, shape, device=gpu).float()
    else:
        x = torch.randn(shape, device=gpu)
    x = x.to(torch.bfloat16).to(memory_format=torch.channels_last).requires_grad_()
    y = stem_maxpool(x)
    assert type(y.grad_fn).__name__ == "_MaxPool3s2Backward"  # the HIP kernels ran, not torch's max_pool2d
    assert y.is_contiguous(memory_format=torch.channels_last)
    g = torch.randint(-4, 5, y.shape, device=gpu).to(torch.bfloat16)  # exact fp32 sums in both backwards
    y.backward(g)
    xt = x.detach().clone().requires_grad_()
    with reference_ops():
        yt = torch.nn.functional.max_pool2d(xt, 3, 2, 1)
    yt.backward(g)
    assert torch.equal(y, yt)
    assert torch.equal(x.grad, xt.grad)


def test_stem_maxpool_propagates_nan_like_torch(gpu):
    """a window holding a NaN outputs NaN even when a larger finite value follows the NaN in
    scan order (torch: `val > max || isnan(val)`; nothing replaces a NaN once held)."""
    from distributedvolunteercomputing_amd.ops.batchnorm import stem_maxpool

    torch.manual_seed(3)
    x = torch.randn(2, 8, 9, 9, device=gpu)
    x[0, :, 2, 2] = float("nan")  # then larger finite values right after it in the same windows
    x[0, :, 2, 3] = 100.0
    x[1, 3, 0, 0] = float("nan")
    x = x.to(torch.bfloat16).to(memory_format=torch.channels_last).requires_grad_()
    y = stem_maxpool(x)
    assert type(y.grad_fn).__name__ == "_MaxPool3s2Backward"
    with reference_ops(), torch.no_grad():
        yt = torch.nn.functional.max_pool2d(x, 3, 2, 1)
    y = y.detach()
    assert torch.equal(torch.isnan(y), torch.isnan(yt)) and bool(torch.isnan(y).any())
    fin = ~torch.isnan(yt)
    assert torch.equal(y[fin], yt[fin])


def test_fused_batchnorm_large_mean_variance(gpu):
    """|mean| >> std over many rows. The statistics are summed around a per-channel pivot
    (a value of the batch), so the variance keeps its digits where E[x^2] - m^2 on raw fp32 sums would
    cancel. Oracle: float64 statistics of the same bf16 input (torch's fp32 BatchNorm itself scatters
    by +-2.5 % per channel on this input, so it is not the reference here)."""
    from distributedvolunteercomputing_amd.ops.batchnorm import bn_act

    torch.manual_seed(11)
    C = 64
    bn = torch.nn.BatchNorm2d(C, momentum=1.0).to(gpu).to(torch.bfloat16)  # running_var = this batch's variance
    # mean 200, std 0.5 (bf16 spacing at 200 is 1.0: the values are the integers 198..202)
    x = (200 + 0.5 * torch.randn(32, C, 56, 56, device=gpu)).to(torch.bfloat16)
    x = x.to(memory_format=torch.channels_last)
    y = bn_act(x, bn, None, relu=False)
    assert type(y.grad_fn).__name__ == "_BNActBackward"
    xd = x.double()
    mean = xd.mean(dim=(0, 2, 3))
    var_b = xd.var(dim=(0, 2, 3), unbiased=False)
    var_u = xd.var(dim=(0, 2, 3), unbiased=True)
    # running stats are bf16 (spacing 2^-9 at 0.33): within that rounding of the float64 oracle
    assert float(((bn.running_var.double() - var_u).abs() / var_u).max()) < 4e-3
    assert float(((bn.running_mean.double() - mean).abs() / mean).max()) < 4e-3
    yd = (xd - mean[None, :, None, None]) / torch.sqrt(var_b[None, :, None, None] + bn.eps)
    yd = yd * bn.weight.double()[None, :, None, None] + bn.bias.double()[None, :, None, None]
    assert float((y.double() - yd).norm() / yd.norm()) < 1e-2


@pytest.mark.parametrize("N,H,C", [(2, 3, 64), (3, 9, 128), (5, 11, 256), (7, 13, 64)])
def test_fused_batchnorm_ragged_row_counts(gpu, N, H, C):
    """The reductions' pipelined row loop (csrc/kernels/batchnorm.hip channel_reduce_pipe) at row counts that leave
    no full group of rows, an odd number of groups, lanes diverging between a full group and the single-row
    tail: output and gradients against torch's BatchNorm + ReLU in fp32."""
    from distributedvolunteercomputing_amd.ops.batchnorm import bn_act

    torch.manual_seed(N * H + C)
    bn = torch.nn.BatchNorm2d(C).to(gpu)
    torch.nn.init.uniform_(bn.weight, 0.5, 1.5)
    torch.nn.init.uniform_(bn.bias, -0.5, 0.5)
    bn32 = torch.nn.BatchNorm2d(C).to(gpu)
    bn32.load_state_dict(bn.state_dict())
    bn = bn.to(torch.bfloat16)
    x = (torch.randn(N, C, H, H, device=gpu) + 0.3).to(torch.bfloat16).to(memory_format=torch.channels_last)
    x.requires_grad_()
    y = bn_act(x, bn, None, True)
    assert type(y.grad_fn).__name__ == "_BNActBackward"
    g = torch.randn_like(y)
    y.backward(g)
    x32 = x.detach().float().requires_grad_()
    y32 = torch.relu(bn32(x32))
    y32.backward(g.float())
    # torch's own bf16 BatchNorm + ReLU sets the bar (a ReLU output's gradients: elements near 0 round to the
    # other side of the mask, as in test_fused_batchnorm_act_vs_fp32)
    bnt = torch.nn.BatchNorm2d(C).to(gpu)
    bnt.load_state_dict(bn32.state_dict())
    bnt = bnt.to(torch.bfloat16)
    xt = x.detach().clone().requires_grad_()
    with reference_ops():
        yt = torch.relu(bnt(xt))
        yt.backward(g)
    rel = lambda a, b: float((a.float() - b).norm() / (b.norm() + 1e-6))  # noqa: E731

    def ok(a, t, ref, tol):
        e, et = rel(a, ref), rel(t, ref)
        assert e < max(tol, 1.1 * et), (e, et)

    ok(y, yt, y32, 1e-2)
    ok(x.grad, xt.grad, x32.grad, 1e-2)
    ok(bn.weight.grad, bnt.weight.grad, bn32.weight.grad, 1e-2)
    ok(bn.bias.grad, bnt.bias.grad, bn32.bias.grad, 1e-2)


@pytest.mark.parametrize("N,H,W,C,s", [(3, 56, 56, 256, 2), (2, 14, 14, 1024, 2), (2, 7, 9, 64, 2), (1, 5, 5, 8, 3)])
def test_nhwc_subsample_kernels_vs_torch(gpu, N, H, W, C, s):
    """The strided-shortcut helpers (csrc/kernels/batchnorm.hip): subsample_nhwc = x[:, ::s, ::s, :],
    subsample_add_nhwc = full[:, ::s, ::s, :] += g (bit-exact: one bf16 add per element, as torch's), and
    bcast_hw_nhwc = g[:, None, None, :] * scale."""
    from distributedvolunteercomputing_amd.ops import native

    C_ = native()
    torch.manual_seed(N * H + C)
    x = torch.randn(N, H, W, C, device=gpu).to(torch.bfloat16)
    y = C_.subsample_nhwc(x, s)
    assert torch.equal(y, x[:, ::s, ::s, :])
    g = torch.randn_like(y)
    full = x.clone()
    ref = x.clone()
    ref[:, ::s, ::s, :].add_(g)
    C_.subsample_add_nhwc(full, g, s)
    assert torch.equal(full, ref)
    gg = torch.randn(N, C, device=gpu).to(torch.bfloat16)
    out = C_.bcast_hw_nhwc(gg, H, W, 1.0 / (H * W))
    refb = (gg.float() / (H * W))[:, None, None, :].expand(N, H, W, C)
    assert (out.float() - refb).abs().max().item() <= 1e-2 * refb.abs().max().item()


def test_global_avgpool_and_subsample_tap_grads(gpu):
    """global_avgpool (HIP broadcast backward) and subsample_tap (HIP subsample forward, strided add backward into
    the deposited conv1 gradient) against torch autograd on the same bf16 inputs."""
    from distributedvolunteercomputing_amd.ops.batchnorm import global_avgpool
    from distributedvolunteercomputing_amd.ops.linear import GradJoin, subsample_tap

    torch.manual_seed(5)
    x = torch.randn(4, 64, 7, 7, device=gpu).to(torch.bfloat16).to(memory_format=torch.channels_last).requires_grad_()
    g = torch.randn(4, 64, device=gpu).to(torch.bfloat16)
    global_avgpool(x).backward(g)
    x2 = x.detach().clone().requires_grad_()
    torch.flatten(torch.nn.functional.adaptive_avg_pool2d(x2, 1), 1).backward(g)
    assert x.grad.is_contiguous(memory_format=torch.channels_last)
    assert (x.grad.float() - x2.grad.float()).abs().max().item() < 1e-3
    # subsample_tap: the stride-2 shortcut's input gradient lands in the buffer conv1 deposited
    xs = torch.randn(2, 32, 9, 11, device=gpu).to(torch.bfloat16).to(memory_format=torch.channels_last)
    xs.requires_grad_()
    join = GradJoin()
    sub = subsample_tap(xs, join, 2)
    assert torch.equal(sub, xs.detach().permute(0, 2, 3, 1)[:, ::2, ::2, :])
    dep = torch.randn(2, 9, 11, 32, device=gpu).to(torch.bfloat16)
    join.pending = dep.reshape(-1, 32).clone()
    gs = torch.randn_like(sub)
    sub.backward(gs)
    ref = dep.clone()
    ref[:, ::2, ::2, :] += gs
    assert torch.equal(xs.grad.permute(0, 2, 3, 1), ref)
