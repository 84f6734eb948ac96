"""Compression kernels (top-k + EF, PowerSGD) on gfx950 vs torch references."""
import pytest
import torch

from distributedvolunteercomputing_amd.models.gpt2 import GPT2, GPT2Config
from distributedvolunteercomputing_amd.ops._lib import reference_ops
from distributedvolunteercomputing_amd.parallel.compression import PowerSGDCompressor, TopKCompressor
from distributedvolunteercomputing_amd.parallel.flat_params import FlatParams

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,ratio", [(1_000_003, 0.01), (65536, 0.1), (4096, 0.5), (777, 0.01), (16_777_219, 0.01)])
def test_topk_exact(gpu, n, ratio):
    torch.manual_seed(0)
    c = TopKCompressor(n, ratio, gpu)
    g = torch.randn(n, device=gpu).to(torch.bfloat16)
    e0 = torch.randn(n, device=gpu) * 0.1
    c.e.copy_(e0)
    acc = g.float() + e0
    idx, val = c.compress(g)
    torch.cuda.synchronize()
    k = c.k
    sel = idx.long()
    assert len(set(sel.tolist())) == k  # distinct
    thr = torch.topk(acc.abs(), k).values[-1]
    assert (acc[sel].abs() >= thr - 1e-6).all()
    assert torch.allclose(val.float(), acc[sel].to(torch.bfloat16).float())
    # error feedback: a selected entry keeps its bf16 rounding residual, the rest is kept whole
    mask = torch.ones(n, dtype=torch.bool, device=gpu)
    mask[sel] = False
    assert torch.equal(c.e[sel], acc[sel] - val.float()) and torch.equal(c.e[mask], acc[mask])
    assert (c.e[sel].abs() <= acc[sel].abs() * 2.0**-8).all()


def test_topk_ties_and_zeros(gpu):
    n = 10000
    c = TopKCompressor(n, 0.05, gpu, value_dtype=torch.float32)
    g = torch.zeros(n, device=gpu)
    g[:100] = 1.0  # 100 tied maxima, k = 500 > number of non-zeros
    idx, val = c.compress(g)
    torch.cuda.synchronize()
    nz = (val != 0).sum().item()
    assert nz == 100 and set(idx[val != 0].tolist()) == set(range(100))


@pytest.mark.parametrize("n", [1_000_003, 4_194_304])
def test_topk_bf16_ties_every_round(gpu, n):
    """bf16 gradients with e = 0 put thousands of elements exactly on the threshold value: the
    tie budget must hand out exactly k - (#above) of them, and the scratch state (histogram,
    claim counter) must be clean for the next round."""
    torch.manual_seed(7)
    c = TopKCompressor(n, 0.01, gpu)
    for rnd in range(3):
        c.e.zero_()
        g = torch.randn(n, device=gpu).to(torch.bfloat16)
        acc = g.float()
        idx, val = c.compress(g)
        torch.cuda.synchronize()
        sel = idx.long()
        assert sel.unique().numel() == c.k, rnd
        thr = torch.topk(acc.abs(), c.k).values[-1]
        above = (acc.abs() > thr).sum().item()
        ties = (acc.abs() == thr).sum().item()
        assert ties > 10, "the test needs ties on the threshold"
        assert (acc[sel].abs() >= thr).all()
        assert (acc[sel].abs() > thr).sum().item() == above  # every element above is selected
        assert torch.equal(val.float(), acc[sel])  # bf16 in, bf16 out: no residual
    assert int(c.hist.abs().sum()) == 0  # left zeroed for the next round


def test_allreduce_mean_packed_wire(gpu):
    """P = 1 path of the packed wire: the bf16 output is the scatter of the selected pairs."""
    torch.manual_seed(8)
    n = 300_001
    c = TopKCompressor(n, 0.02, gpu)
    g = torch.randn(n, device=gpu).to(torch.bfloat16)
    out = c.allreduce_mean(g, None)
    torch.cuda.synchronize()
    ref = torch.zeros(n, device=gpu)
    ref[c.idx.long()] = c.val.float()
    assert torch.equal(out.float(), ref.to(torch.bfloat16).float())
    assert out.data_ptr() == c.allreduce_mean(g, None).data_ptr()  # preallocated, reused


def test_scatter_add_packed_drops_bad_indices(gpu):
    from distributedvolunteercomputing_amd.ops import native

    k = 3
    wire = torch.zeros(2, k + 2, dtype=torch.int32, device=gpu)  # bf16 values: 2 words for 3 values
    wire[0, :k] = torch.tensor([1, 7, 1 << 30], dtype=torch.int32)  # the last index is out of range
    wire[0, k:].view(torch.bfloat16)[:k] = torch.tensor([1.0, 2.0, 5.0], dtype=torch.bfloat16)
    wire[1, :k] = torch.tensor([7, -3, 0], dtype=torch.int32)
    wire[1, k:].view(torch.bfloat16)[:k] = torch.tensor([4.0, 8.0, 0.0], dtype=torch.bfloat16)
    dense = torch.zeros(10, device=gpu)
    native().scatter_add_packed(wire, k, True, 0.5, dense)
    torch.cuda.synchronize()
    exp = torch.zeros(10, device=gpu)
    exp[1], exp[7] = 0.5, 3.0
    assert torch.equal(dense, exp)


def test_scatter_add(gpu):
    from distributedvolunteercomputing_amd.ops import native

    dense = torch.zeros(100, device=gpu)
    idx = torch.tensor([1, 5, 1, 99], dtype=torch.int32, device=gpu)
    val = torch.tensor([1.0, 2.0, 3.0, 4.0], device=gpu)
    native().scatter_add(idx, val, 0.5, dense)
    assert dense[1].item() == 2.0 and dense[5].item() == 1.0 and dense[99].item() == 2.0


def test_powersgd_matches_reference(gpu):
    torch.manual_seed(1)
    cfg = GPT2Config.preset("gpt2-tiny")
    m = GPT2(cfg).to(gpu, torch.bfloat16)
    flat = FlatParams(m)
    c_gpu = PowerSGDCompressor(flat, rank=4, device=gpu, seed=3)
    c_ref = PowerSGDCompressor(flat, rank=4, device=gpu, seed=3)
    assert c_gpu.mats and c_gpu.compression_ratio > 2
    for step in range(3):
        g = (torch.randn(flat.numel, device=gpu) * 0.01).to(torch.bfloat16)
        out = c_gpu.allreduce_mean(g, None).float().clone()
        with reference_ops():
            ref = c_ref.allreduce_mean(g, None).float().clone()
        rel = (out - ref).norm() / ref.norm()
        assert rel < 2e-2, (step, float(rel))
        assert (c_gpu.ef() - c_ref.ef()).norm() / (c_ref.ef().norm() + 1e-9) < 2e-2
    # P columns orthonormal after orth
    off, r, cc = c_gpu.mats[0]
    P = c_gpu.P[: r * 4].view(r, 4)
    assert torch.allclose(P.t() @ P, torch.eye(4, device=gpu), atol=1e-3)


def test_powersgd_error_feedback_converges(gpu):
    """A fixed gradient is transmitted exactly in the long run (EF telescopes)."""
    torch.manual_seed(2)
    cfg = GPT2Config.preset("gpt2-tiny")
    m = GPT2(cfg).to(gpu, torch.bfloat16)
    flat = FlatParams(m)
    c = PowerSGDCompressor(flat, rank=4, device=gpu)
    g = (torch.randn(flat.numel, device=gpu) * 0.01).to(torch.bfloat16)
    total = torch.zeros(flat.numel, device=gpu)
    rels = {}
    for t in range(1, 81):
        total += c.allreduce_mean(g, None).float()
        if t in (10, 80):
            rels[t] = float((total / t - g.float()).norm() / g.float().norm())
    # e stays bounded, so the time-averaged transmitted gradient converges to g
    assert rels[80] < 0.5 * rels[10], rels


@pytest.mark.parametrize("rank", [1, 4, 8])
def test_powersgd_odd_shapes_match_reference(gpu, rank):
    """Matrices whose row length is not a multiple of 4 take the scalar paths of the fused
    e += g / P = e Q, Q = e^T P and reconstruct kernels; 4-aligned ones the 16-B paths (with a
    row count that is not a multiple of the 64-row slab and columns past one 1024-column chunk)."""
    torch.manual_seed(4)
    m = torch.nn.Sequential(torch.nn.Linear(67, 131), torch.nn.Linear(131, 1100), torch.nn.Linear(1100, 97))
    m = m.to(gpu, torch.bfloat16)
    flat = FlatParams(m)
    c_gpu = PowerSGDCompressor(flat, rank=rank, device=gpu, seed=5)
    c_ref = PowerSGDCompressor(flat, rank=rank, device=gpu, seed=5)
    assert len(c_gpu.mats) == 3 and any(cc % 4 for _, _, cc in c_gpu.mats)
    for step in range(3):
        g = (torch.randn(flat.numel, device=gpu) * 0.01).to(torch.bfloat16)
        out = c_gpu.allreduce_mean(g, None).float().clone()
        with reference_ops():
            ref = c_ref.allreduce_mean(g, None).float().clone()
        rel = (out - ref).norm() / ref.norm()
        assert rel < 2e-2, (step, float(rel))
        assert (c_gpu.ef() - c_ref.ef()).norm() / (c_ref.ef().norm() + 1e-9) < 2e-2


@pytest.mark.parametrize("rank", [1, 2, 4, 8])
def test_psgd_orth_equals_thin_qr(gpu, rank):
    """Batched CholeskyQR2 of every matrix's P (rows spanning several 2048-row slabs) equals the
    thin-QR factor with a positive-diagonal R (the unique orthonormalisation Gram-Schmidt gives)."""
    from distributedvolunteercomputing_amd.ops import native

    torch.manual_seed(10 + rank)
    m = torch.nn.Sequential(torch.nn.Linear(300, 5000, bias=False), torch.nn.Linear(5000, 70, bias=False),
                            torch.nn.Linear(64, 9000, bias=False)).to(gpu, torch.bfloat16)
    flat = FlatParams(m)
    c = PowerSGDCompressor(flat, rank=rank, device=gpu)
    assert len(c.mats) == 3
    c.P.copy_(torch.randn_like(c.P))
    before = c.P.clone()
    native().psgd_orth(c.d_orth, len(c.mats), c.nb_orth, c.P, c.G, rank)
    torch.cuda.synchronize()
    for i, (off, r, cc) in enumerate(c.mats):
        p0 = before[c.p_off[i]: c.p_off[i] + r * rank].view(r, rank).double()
        q, rr = torch.linalg.qr(p0)
        q = q * torch.sign(torch.diagonal(rr)).unsqueeze(0)
        got = c.P[c.p_off[i]: c.p_off[i] + r * rank].view(r, rank).double()
        assert torch.allclose(got, q, atol=2e-5), (i, float((got - q).abs().max()))


def test_psgd_orth_dependent_column_stays_finite(gpu):
    from distributedvolunteercomputing_amd.ops import native

    m = torch.nn.Sequential(torch.nn.Linear(512, 4096, bias=False)).to(gpu, torch.bfloat16)
    c = PowerSGDCompressor(FlatParams(m), rank=4, device=gpu)
    P = c.P[: 4096 * 4].view(4096, 4)
    P.copy_(torch.randn(4096, 4, device=gpu))
    P[:, 2] = P[:, 0] * 3.0  # linearly dependent column
    native().psgd_orth(c.d_orth, len(c.mats), c.nb_orth, c.P, c.G, 4)
    torch.cuda.synchronize()
    # the dependent column's fp32 residual is rounding noise: it becomes SOME unit vector
    # orthogonal to the others (the second CholeskyQR pass cleans it up) — never NaN/inf
    assert torch.isfinite(P).all()
    assert torch.allclose(P.t() @ P, torch.eye(4, device=gpu), atol=1e-3)
