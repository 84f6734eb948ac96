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


def test_llama_sharded_powersgd_trains(gpu):
    cfg = LlamaConfig.preset("llama-tiny")
    m = Llama(cfg).to(gpu, torch.bfloat16)
    tr = ShardedDPTrainer(m, ShardedConfig(lr=3e-3, weight_decay=0.0), device=gpu)
    tr.compressor = PowerSGDCompressor(tr.flat, rank=4, device=gpu)
    x = torch.randint(0, cfg.vocab_size, (4, 64), device=gpu)
    losses = [float(tr.step(x, x.roll(-1, 1))) for _ in range(25)]
    assert losses[-1] < losses[0] - 0.5, losses


def test_resnet_tiny_step(gpu):
    from distributedvolunteercomputing_amd.parallel.compression import TopKCompressor
    from distributedvolunteercomputing_amd.parallel.local_sgd import LocalSGDConfig, LocalSGDTrainer

    m = resnet_tiny().to(gpu, torch.bfloat16).to(memory_format=torch.channels_last)
    tr = LocalSGDTrainer(m, LocalSGDConfig(H=2, lr=1e-3), device=gpu)
    tr.compressor = TopKCompressor(tr.flat.numel, 0.05, gpu)
    x = torch.randn(8, 3, 32, 32, device=gpu).to(torch.bfloat16).to(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,), device=gpu)
    for _ in range(4):
        st = tr.step(x, y)
    torch.cuda.synchronize()
    assert torch.isfinite(st.extra["loss_t"]).item()


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
