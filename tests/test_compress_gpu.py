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
