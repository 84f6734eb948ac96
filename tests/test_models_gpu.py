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
