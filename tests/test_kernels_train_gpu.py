"""Numerics of the training-path HIP kernels vs plain PyTorch fp32 references (gfx950)."""
import pytest
import torch
import torch.nn.functional as F

from distributedvolunteercomputing_amd import ops
from distributedvolunteercomputing_amd.ops import optim as optim_ops

pytestmark = pytest.mark.gpu


def _bf(x):
    return x.to(torch.bfloat16)


@pytest.mark.parametrize("C,R", [(64, 257), (768, 257), (768, 24577), (1024, 257), (1600, 257), (4096, 257)])
@pytest.mark.parametrize("fused", [False, True])
def test_add_layernorm_fwd_bwd(gpu, C, R, fused):
    """R = 24577 at C = 768: every wave of the 768-block backward grid walks many rows."""
    torch.manual_seed(0)
    a = _bf(torch.randn(R, C, device=gpu)).requires_grad_()
    b = _bf(torch.randn(R, C, device=gpu)).requires_grad_() if fused else None
    w = _bf(torch.rand(C, device=gpu) + 0.5).requires_grad_()
    bias = _bf(torch.randn(C, device=gpu) * 0.1).requires_grad_()
    y, x = ops.add_layernorm(a, b, w, bias)
    # reference in fp32 on the bf16-rounded residual
    a32 = a.detach().float().requires_grad_()
    b32 = b.detach().float().requires_grad_() if fused else None
    w32 = w.detach().float().requires_grad_()
    bias32 = bias.detach().float().requires_grad_()
    xr = a32 + b32 if fused else a32
    yr = F.layer_norm(xr, (C,), w32, bias32, 1e-5)
    assert torch.allclose(x.float(), xr.detach(), atol=2e-2, rtol=1e-2)
    assert torch.allclose(y.float(), yr.detach(), atol=3e-2, rtol=2e-2)
    # bf16-representable upstream gradients: the kernel and the reference see the same values
    dy = _bf(torch.randn(R, C, device=gpu)).float()
    dx_res = _bf(torch.randn(R, C, device=gpu)).float()
    loss = (y.float() * dy).sum() + (x.float() * dx_res).sum()
    loss.backward()
    lr = (yr * dy).sum() + (xr * dx_res).sum()
    lr.backward()
    assert torch.allclose(a.grad.float(), a32.grad, atol=5e-2, rtol=3e-2)
    if fused:
        assert torch.allclose(b.grad.float(), b32.grad, atol=5e-2, rtol=3e-2)
    # column sums over R rows: the bf16 rounding of x / y in the forward adds noise ~ sqrt(R)
    tol = 0.5 * max(1.0, (R / 257) ** 0.5)
    assert torch.allclose(w.grad.float(), w32.grad, atol=tol, rtol=3e-2)
    assert torch.allclose(bias.grad.float(), bias32.grad, atol=tol, rtol=3e-2)


def test_rmsnorm(gpu):
    torch.manual_seed(1)
    R, C = 100, 4096
    x = _bf(torch.randn(R, C, device=gpu)).requires_grad_()
    w = _bf(torch.rand(C, device=gpu) + 0.5).requires_grad_()
    y = ops.rmsnorm(x, w)
    x32 = x.detach().float().requires_grad_()
    w32 = w.detach().float().requires_grad_()
    yr = x32 * torch.rsqrt(x32.pow(2).mean(-1, keepdim=True) + 1e-6) * w32
    assert torch.allclose(y.float(), yr, atol=3e-2, rtol=2e-2)
    dy = torch.randn(R, C, device=gpu)
    (y.float() * dy).sum().backward()
    (yr * dy).sum().backward()
    assert torch.allclose(x.grad.float(), x32.grad, atol=5e-2, rtol=3e-2)
    assert torch.allclose(w.grad.float(), w32.grad, atol=0.5, rtol=3e-2)


def test_gelu(gpu):
    torch.manual_seed(2)
    x = _bf(torch.randn(64, 3072, device=gpu) * 3).requires_grad_()
    y = ops.gelu(x)
    x32 = x.detach().float().requires_grad_()
    yr = F.gelu(x32, approximate="tanh")
    assert torch.allclose(y.float(), yr, atol=2e-2, rtol=1e-2)
    dy = torch.randn_like(x32)
    (y.float() * dy).sum().backward()
    (yr * dy).sum().backward()
    assert torch.allclose(x.grad.float(), x32.grad, atol=3e-2, rtol=2e-2)


def test_swiglu(gpu):
    torch.manual_seed(3)
    gu = _bf(torch.randn(33, 2 * 512, device=gpu) * 2).requires_grad_()
    y = ops.swiglu(gu)
    g32 = gu.detach().float().requires_grad_()
    g, u = g32.chunk(2, -1)
    yr = F.silu(g) * u
    assert torch.allclose(y.float(), yr, atol=3e-2, rtol=2e-2)
    dy = torch.randn_like(yr)
    (y.float() * dy).sum().backward()
    (yr * dy).sum().backward()
    assert torch.allclose(gu.grad.float(), g32.grad, atol=5e-2, rtol=3e-2)


@pytest.mark.parametrize("V,Vp", [(50257, 50304), (1000, 1000), (37, 40), (128256, 128256)])
def test_cross_entropy(gpu, V, Vp):
    torch.manual_seed(4)
    R = 129
    logits = _bf(torch.randn(R, Vp, device=gpu) * 3).requires_grad_()
    tgt = torch.randint(0, V, (R,), device=gpu)
    tgt[5] = -100
    loss = ops.cross_entropy(logits * 1.0, tgt, vocab=V)
    l32 = logits.detach().float().requires_grad_()
    ref = F.cross_entropy(l32[:, :V], tgt, ignore_index=-100)
    assert abs(loss.item() - ref.item()) < 2e-3 * max(1.0, abs(ref.item()))
    (loss * 2.0).backward()
    (ref * 2.0).backward()
    assert torch.allclose(logits.grad.float(), l32.grad, atol=2e-4, rtol=2e-2)
    if Vp > V:
        assert logits.grad[:, V:].abs().max().item() == 0.0


@pytest.mark.parametrize("max_norm", [0.0, 1.0])
def test_adamw_flat_matches_reference(gpu, max_norm):
    torch.manual_seed(5)
    n = 64 * 1000 + 8
    n_decay = 64 * 600
    p = _bf(torch.randn(n, device=gpu))
    g = _bf(torch.randn(n, device=gpu) * 0.1)
    master = p.float()
    m = torch.zeros(n, device=gpu)
    v = torch.zeros(n, device=gpu)
    st = ops.new_ostate(gpu, 1e-2)
    # CPU reference copies
    pc, gc, mc, m2, v2 = p.cpu(), g.cpu(), master.cpu(), m.cpu(), v.cpu()
    stc = st.cpu()
    for _ in range(3):
        ops.adamw_step(p, g, master, m, v, st, n_decay=n_decay, beta1=0.9, beta2=0.95, eps=1e-8, wd=0.1,
                       max_norm=max_norm)
        optim_ops.adamw_step(pc, gc, mc, m2, v2, stc, n_decay=n_decay, beta1=0.9, beta2=0.95, eps=1e-8, wd=0.1,
                             max_norm=max_norm)
    torch.cuda.synchronize()
    assert st[0].item() == 3
    assert torch.allclose(master.cpu(), mc, atol=1e-5, rtol=1e-5)
    assert torch.allclose(m.cpu(), m2, atol=1e-6, rtol=1e-5)
    assert torch.allclose(v.cpu(), v2, atol=1e-7, rtol=1e-5)
    assert torch.allclose(p.cpu().float(), mc.to(torch.bfloat16).float(), atol=1e-2, rtol=1e-2)
    if max_norm > 0:
        assert abs(st[2].item() - stc[2].item()) < 1e-4


def test_lsgd_delta_apply(gpu):
    torch.manual_seed(6)
    n = 64 * 77
    master = torch.randn(n, device=gpu)
    anchor = master + torch.randn(n, device=gpu) * 1e-2
    delta = torch.empty(n, dtype=torch.bfloat16, device=gpu)
    ops.lsgd_delta(master, anchor, delta)
    assert torch.allclose(delta.float(), master - anchor, atol=1e-4, rtol=1e-2)
    param = torch.empty(n, dtype=torch.bfloat16, device=gpu)
    mom = torch.zeros(n, device=gpu)
    a0 = anchor.clone()
    ops.lsgd_apply(delta, anchor, master, param, mom, outer_lr=0.7, mu=0.9, nesterov=True, avg_scale=0.5)
    gref = -delta.float() * 0.5
    momr = gref
    upd = gref + 0.9 * momr
    ar = a0 - 0.7 * upd
    assert torch.allclose(anchor, ar, atol=1e-6, rtol=1e-5)
    assert torch.equal(master, anchor)
    assert torch.equal(param, anchor.to(torch.bfloat16))
    assert torch.allclose(mom, momr)


def test_axpy_bf16(gpu):
    a = _bf(torch.randn(4096, device=gpu))
    b = _bf(torch.randn(4096, device=gpu))
    ref = (a.float() + 0.5 * b.float()).to(torch.bfloat16)
    ops.axpy_bf16(b, a, 0.5)
    assert torch.equal(a, ref)


def test_add_layernorm_branch_bias(gpu):
    torch.manual_seed(7)
    R, C = 300, 768
    a = _bf(torch.randn(R, C, device=gpu)).requires_grad_()
    b = _bf(torch.randn(R, C, device=gpu)).requires_grad_()
    bb = _bf(torch.randn(C, device=gpu)).requires_grad_()
    w = _bf(torch.rand(C, device=gpu) + 0.5).requires_grad_()
    y, x = ops.add_layernorm(a, b, w, None, branch_bias=bb)
    a32, b32, bb32, w32 = (t.detach().float().requires_grad_() for t in (a, b, bb, w))
    xr = a32 + b32 + bb32
    yr = F.layer_norm(xr, (C,), w32, None, 1e-5)
    assert torch.allclose(y.float(), yr, atol=3e-2, rtol=2e-2)
    dy, dxr = torch.randn(R, C, device=gpu), torch.randn(R, C, device=gpu)
    ((y.float() * dy).sum() + (x.float() * dxr).sum()).backward()
    ((yr * dy).sum() + (xr * dxr).sum()).backward()
    assert torch.allclose(bb.grad.float(), bb32.grad, atol=0.5, rtol=3e-2)
    assert torch.allclose(b.grad.float(), b32.grad, atol=5e-2, rtol=3e-2)


@pytest.mark.parametrize("R", [1000, 9001])
def test_bias_gelu(gpu, R):
    """R = 9001: each row group runs the pipelined 4-row steps and the row tail."""
    torch.manual_seed(8)
    x = _bf(torch.randn(R, 3072, device=gpu) * 2).requires_grad_()
    b = _bf(torch.randn(3072, device=gpu)).requires_grad_()
    y = ops.bias_gelu(x, b)
    x32, b32 = x.detach().float().requires_grad_(), b.detach().float().requires_grad_()
    yr = F.gelu(x32 + b32, approximate="tanh")
    assert torch.allclose(y.float(), yr, atol=3e-2, rtol=2e-2)
    dy = _bf(torch.randn_like(yr)).float()
    (y.float() * dy).sum().backward()
    (yr * dy).sum().backward()
    assert torch.allclose(x.grad.float(), x32.grad, atol=5e-2, rtol=3e-2)
    assert torch.allclose(b.grad.float(), b32.grad, atol=1.0 * max(1.0, (R / 1000) ** 0.5), rtol=3e-2)


def test_embedding_fwd_bwd(gpu):
    torch.manual_seed(9)
    V, C, B, T = 1000, 768, 4, 100
    idx = torch.randint(0, V, (B, T), device=gpu)
    wte = _bf(torch.randn(V, C, device=gpu)).requires_grad_()
    wpe = _bf(torch.randn(128, C, device=gpu)).requires_grad_()
    x = ops.embed(idx, wte, wpe)
    w32, p32 = wte.detach().float().requires_grad_(), wpe.detach().float().requires_grad_()
    xr = F.embedding(idx, w32) + p32[:T]
    assert torch.allclose(x.float(), xr, atol=2e-2, rtol=1e-2)
    dy = torch.randn_like(xr)
    (x.float() * dy).sum().backward()
    (xr * dy).sum().backward()
    assert torch.allclose(wte.grad.float(), w32.grad, atol=5e-2, rtol=2e-2)
    assert torch.allclose(wpe.grad.float(), p32.grad, atol=5e-2, rtol=2e-2)


# (4096, 4096, 4096): a big output at few tokens (the Llama-3-8B shape) takes the single
# beta = 1 GEMM into .grad instead of the split-M batch
@pytest.mark.parametrize("M,N,K,bias", [(8192, 768, 768, True), (65536, 2304, 768, False), (4096, 512, 96, False),
                                        (4096, 4096, 4096, False)])
@pytest.mark.parametrize("preset_grad", [False, True])
def test_linear_splitm_wgrad(gpu, M, N, K, bias, preset_grad):
    """ops.linear: split-M batched weight gradient (HIP fp32 reduction into .grad) against an
    fp32 reference; with a preset .grad (the flat-buffer case) the gradient is accumulated."""
    torch.manual_seed(0)
    x = torch.randn(M, K, device=gpu).to(torch.bfloat16).requires_grad_()
    w = (torch.randn(N, K, device=gpu) * 0.05).to(torch.bfloat16).requires_grad_()
    b = torch.randn(N, device=gpu).to(torch.bfloat16).requires_grad_() if bias else None
    g0 = torch.randn(N, K, device=gpu).to(torch.bfloat16)
    if preset_grad:
        w.grad = g0.clone()
    dy = torch.randn(M, N, device=gpu).to(torch.bfloat16)
    y = ops.linear(x, w, b)
    y.backward(dy)
    xr, wr = x.detach().float().requires_grad_(), w.detach().float().requires_grad_()
    br = b.detach().float().requires_grad_() if bias else None
    F.linear(xr, wr, br).backward(dy.float())
    ref_w = wr.grad + (g0.float() if preset_grad else 0)
    rel = lambda a, r: float((a.float() - r).norm() / r.norm())  # noqa: E731
    assert rel(y, F.linear(xr, wr, br)) < 1e-2
    assert rel(x.grad, xr.grad) < 1e-2
    assert rel(w.grad, ref_w) < 1e-2, rel(w.grad, ref_w)
    if bias:
        assert rel(b.grad, br.grad) < 1e-2


def test_layernorm_grads_accumulate_into_preset_buffers(gpu):
    """With preset .grad buffers (the flat-buffer case) the LN parameter gradients are ADDED into
    them by the HIP column sums (autograd gets None for those inputs)."""
    torch.manual_seed(11)
    R, C = 513, 768
    a = _bf(torch.randn(R, C, device=gpu)).requires_grad_()
    b = _bf(torch.randn(R, C, device=gpu)).requires_grad_()
    w = _bf(torch.rand(C, device=gpu) + 0.5).requires_grad_()
    bias = _bf(torch.randn(C, device=gpu) * 0.1).requires_grad_()
    bb = _bf(torch.randn(C, device=gpu)).requires_grad_()
    g0 = {n: _bf(torch.randn(C, device=gpu)) for n in ("w", "bias", "bb")}
    w.grad, bias.grad, bb.grad = g0["w"].clone(), g0["bias"].clone(), g0["bb"].clone()
    y, x = ops.add_layernorm(a, b, w, bias, branch_bias=bb)
    dy, dxr = torch.randn(R, C, device=gpu), torch.randn(R, C, device=gpu)
    ((y.float() * dy).sum() + (x.float() * dxr).sum()).backward()
    a32, b32, w32, bias32, bb32 = (t.detach().float().requires_grad_() for t in (a, b, w, bias, bb))
    xr = a32 + b32 + bb32
    yr = F.layer_norm(xr, (C,), w32, bias32, 1e-5)
    ((yr * dy).sum() + (xr * dxr).sum()).backward()
    for p, r, n in ((w, w32, "w"), (bias, bias32, "bias"), (bb, bb32, "bb")):
        ref = r.grad + g0[n].float()
        assert float((p.grad.float() - ref).norm() / ref.norm()) < 1e-2, n
    assert float((a.grad.float() - a32.grad).norm() / a32.grad.norm()) < 2e-2


@pytest.mark.parametrize("R,F_", [(65536, 2304), (1000, 768), (7, 64)])
def test_colsum_bf16(gpu, R, F_):
    torch.manual_seed(12)
    y = _bf(torch.randn(R, F_, device=gpu))
    C = ops.native()
    out = C.colsum_bf16(y)
    ref = y.float().sum(0)
    assert float((out.float() - ref).norm() / ref.norm()) < 1e-2
    acc = _bf(torch.randn(F_, device=gpu))
    ref2 = ref + acc.float()
    C.colsum_bf16(y, acc)
    assert float((acc.float() - ref2).norm() / ref2.norm()) < 1e-2


def test_embedding_grads_accumulate_into_preset_buffers(gpu):
    torch.manual_seed(13)
    V, C, B, T = 1000, 768, 8, 100
    idx = torch.randint(0, V, (B, T), device=gpu)
    wte = _bf(torch.randn(V, C, device=gpu)).requires_grad_()
    wpe = _bf(torch.randn(128, C, device=gpu)).requires_grad_()
    g_te, g_pe = _bf(torch.randn(V, C, device=gpu)), _bf(torch.randn(128, C, device=gpu))
    wte.grad, wpe.grad = g_te.clone(), g_pe.clone()
    x = ops.embed(idx, wte, wpe)
    dy = torch.randn(B, T, C, device=gpu)
    (x.float() * dy).sum().backward()
    w32, p32 = wte.detach().float().requires_grad_(), wpe.detach().float().requires_grad_()
    (((F.embedding(idx, w32) + p32[:T]) * dy).sum()).backward()
    assert torch.allclose(wte.grad.float(), w32.grad + g_te.float(), atol=6e-2, rtol=2e-2)
    assert torch.allclose(wpe.grad.float(), p32.grad + g_pe.float(), atol=2e-1, rtol=2e-2)


@pytest.mark.parametrize("P,n", [(2, 64), (5, 4104), (8, 31 * 1024 * 8)])
def test_reduce_bcast_bf16_vs_fp32(gpu, P, n):
    """Direct all-reduce middle step: sum of P received shard copies, written to every row of the
    (aliased) send buffer and to this peer's own shard."""
    torch.manual_seed(P)
    inp = _bf(torch.randn(P * n, device=gpu))
    ref = inp.float().view(P, n).sum(0)
    mine = torch.empty(n, device=gpu, dtype=torch.bfloat16)
    ops.reduce_bcast_bf16(inp, inp, mine, P)  # out aliases inp, as in collectives._direct
    torch.cuda.synchronize()
    assert ops.native() is not None
    tol = 2e-2 * ref.abs().max().item()
    assert (mine.float() - ref).abs().max().item() < tol
    for r in range(P):
        assert torch.equal(inp.view(P, n)[r], mine)


@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (512, 768, 192), (1024, 512, 768), (768, 3072, 256)])
@pytest.mark.parametrize("epi", [0, 1, 2, 3])
def test_gemm_nt_epilogues_vs_fp32(gpu, M, N, K, epi):
    """Hand-written MFMA GEMM (gemm.hip) against an fp32 torch reference, every epilogue."""
    C = ops.native()
    torch.manual_seed(M + N + K + epi)
    a = _bf(torch.randn(M, K, device=gpu))
    b = _bf(torch.randn(N, K, device=gpu) * 0.05)
    bias = _bf(torch.randn(N, device=gpu) * 0.1)
    c = torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    c2 = _bf(torch.randn(M, N, device=gpu)) if epi == 3 else torch.empty(M, N, device=gpu, dtype=torch.bfloat16)
    pre_in = c2.clone()
    cs = torch.zeros(N, device=gpu, dtype=torch.float32)
    C.gemm_nt(a, b, c, c2, bias, cs, epi)
    ref = a.float() @ b.float().t()
    if epi == 1:
        ref = ref + bias.float()
    elif epi == 2:
        ref = ref + bias.float()
        g = F.gelu(ref, approximate="tanh")
        assert (c2.float() - g).abs().max() < 2e-2 * g.abs().max()
    elif epi == 3:
        x = pre_in.float().requires_grad_()
        F.gelu(x, approximate="tanh").backward(ref)
        ref = x.grad
        colsum = c.float().sum(0)
        assert (cs - colsum).abs().max() < 1e-2 * colsum.abs().max() + 1e-3
    assert (c.float() - ref).abs().max() < 2e-2 * ref.abs().max()


def test_mlp_gelu_fused_matches_unfused(gpu):
    """ops.mlp_gelu on the hand-written GEMM (VCX_GEMM=vcx) vs the library + bias_gelu path."""
    torch.manual_seed(0)
    x = _bf(torch.randn(512, 768, device=gpu))
    w1 = _bf(torch.randn(3072, 768, device=gpu) * 0.02).requires_grad_()
    b1 = _bf(torch.randn(3072, device=gpu) * 0.02).requires_grad_()
    w2 = _bf(torch.randn(768, 3072, device=gpu) * 0.02).requires_grad_()
    dy = _bf(torch.randn(512, 768, device=gpu))
    outs = {}
    for backend in ("lib", "vcx"):
        ops.set_gemm_backend(backend)
        xi = x.clone().requires_grad_()
        for p in (w1, b1, w2):
            p.grad = None
        y = ops.mlp_gelu(xi, w1, b1, w2)
        y.backward(dy)
        outs[backend] = [t.float().clone() for t in (y, xi.grad, w1.grad, b1.grad, w2.grad)]
    ops.set_gemm_backend("lib")
    for a, b in zip(outs["lib"], outs["vcx"]):
        assert (a - b).norm() / b.norm() < 2e-2




@pytest.mark.parametrize("R,Cc", [(768, 2304), (2304, 768), (3072, 768), (72, 40), (100, 36)])
def test_transpose_bf16(gpu, R, Cc):
    """W -> W^T for the input-gradient GEMM: the 16-B vector kernel (R, Cc multiples of 8, edge tiles
    included) and the element kernel (other shapes), bitwise against torch."""
    w = torch.randn(R, Cc, device=gpu).to(torch.bfloat16)
    t = ops.native().transpose_bf16(w)
    assert torch.equal(t, w.t().contiguous())


@pytest.mark.parametrize("grad_fwd", [True, False])
def test_mlp_gelu_persistent_matches_unfused(gpu, grad_fwd):
    """ops.mlp_gelu on gemm_ps (the default fused MLP) vs the library + bias_gelu path, with gelu'(pre)
    stored by the forward (epilogues 5 / 6, the round-6 default) and with pre stored (epilogues 2 / 4);
    gradients of every input compared as a whole."""
    from distributedvolunteercomputing_amd import config

    torch.manual_seed(1)
    x = _bf(torch.randn(1024, 768, device=gpu))
    w1 = _bf(torch.randn(3072, 768, device=gpu) * 0.02).requires_grad_()
    b1 = _bf(torch.randn(3072, device=gpu) * 0.02).requires_grad_()
    w2 = _bf(torch.randn(768, 3072, device=gpu) * 0.02).requires_grad_()
    dy = _bf(torch.randn(1024, 768, device=gpu))
    outs = {}
    for mode in ("lib", "fused"):
        with config.override(mlp=mode, mlp_grad_fwd=grad_fwd):
            xi = x.clone().requires_grad_()
            for p in (w1, b1, w2):
                p.grad = None
            y = ops.mlp_gelu(xi, w1, b1, w2)
            y.backward(dy)
            outs[mode] = [t.float().clone() for t in (y, xi.grad, w1.grad, b1.grad, w2.grad)]
    for a, b in zip(outs["lib"], outs["fused"]):
        assert (a - b).norm() / b.norm() < 2e-2


def test_mlp_gelu_bias_grad_into_flat_buffer_repeats(gpu):
    """The fused MLP's fc bias gradient added into a preset .grad buffer (the flat-parameter path) through the
    zero-at-rest column-sum buffer (ops/linear.py _colsum_buffer): three backwards accumulate 3x the gradient the
    returned-tensor path gives once, and the buffer is left zeroed."""
    import importlib

    L = importlib.import_module("distributedvolunteercomputing_amd.ops.linear")  # the module, not ops.linear()
    torch.manual_seed(3)
    x = _bf(torch.randn(512, 768, device=gpu))
    w1 = _bf(torch.randn(3072, 768, device=gpu) * 0.02).requires_grad_()
    b1 = _bf(torch.randn(3072, device=gpu) * 0.02).requires_grad_()
    w2 = _bf(torch.randn(768, 3072, device=gpu) * 0.02).requires_grad_()
    dy = _bf(torch.randn(512, 768, device=gpu))
    ops.mlp_gelu(x, w1, b1, w2).backward(dy)  # b1.grad None: the sums come back as a tensor
    ref = b1.grad.float().clone()
    b1.grad = torch.zeros_like(b1)  # a preset buffer: grad_buffer() path
    for _ in range(3):
        ops.mlp_gelu(x, w1, b1, w2).backward(dy)
    torch.cuda.synchronize()
    assert (b1.grad.float() - 3 * ref).norm() / (3 * ref).norm() < 2e-2
    bufs = [v for k, v in L._COLSUM.items() if k[0] == 3072]
    assert bufs and all(int(torch.count_nonzero(v)) == 0 for v in bufs)


@pytest.mark.parametrize("use", ["y", "x"])
def test_add_layernorm_one_output_unused(gpu, use):
    """add_layernorm with only one of its outputs used (GPT-2's last block leaves the residual stream unused): no
    zero-filled gradient is materialised for the other, and the gradients match fp32 (branch bias included)."""
    torch.manual_seed(4)
    R, C = 513, 768
    a = _bf(torch.randn(R, C, device=gpu)).requires_grad_()
    b = _bf(torch.randn(R, C, device=gpu)).requires_grad_()
    w = _bf(torch.rand(C, device=gpu) + 0.5).requires_grad_()
    bias = _bf(torch.randn(C, device=gpu) * 0.1).requires_grad_()
    bb = _bf(torch.randn(C, device=gpu) * 0.1).requires_grad_()
    y, x = ops.add_layernorm(a, b, w, bias, branch_bias=bb)
    g = _bf(torch.randn(R, C, device=gpu)).float()
    ((y if use == "y" else x).float() * g).sum().backward()
    a32, b32, w32, bias32, bb32 = (t.detach().float().requires_grad_() for t in (a, b, w, bias, bb))
    xr = a32 + b32 + bb32
    yr = F.layer_norm(xr, (C,), w32, bias32, 1e-5)
    ((yr if use == "y" else xr) * g).sum().backward()
    assert torch.allclose(a.grad.float(), a32.grad, atol=5e-2, rtol=3e-2)
    assert torch.allclose(b.grad.float(), b32.grad, atol=5e-2, rtol=3e-2)
    assert (bb.grad.float() - bb32.grad).norm() / bb32.grad.norm() < 2e-2
    if use == "y":
        assert (w.grad.float() - w32.grad).norm() / w32.grad.norm() < 2e-2
    else:
        assert w.grad is None or float(w.grad.float().abs().max()) == 0.0
