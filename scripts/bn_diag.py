"""Numerics of the fused train-mode BatchNorm (+ residual) (+ ReLU) against fp32, next to the plain
torch bf16 path's own error on the same inputs; then the ResNet bottleneck oracle comparison
(tests/test_models_gpu.py::_oracle_compare) per path (fused BN / torch BN x 1x1-GEMM / MIOpen 1x1)
and seed: which component moves which gradient."""
import copy
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedvolunteercomputing_amd import config  # noqa: E402
from distributedvolunteercomputing_amd.models.resnet import resnet_tiny  # noqa: E402
from distributedvolunteercomputing_amd.ops._lib import reference_ops  # noqa: E402
from distributedvolunteercomputing_amd.ops.batchnorm import bn_act  # noqa: E402

dev = torch.device("cuda", 0)
rel = lambda a, b: float((a.float() - b).norm() / (b.norm() + 1e-6))  # noqa: E731

print("== fused BN vs fp32 (torch bf16 path's error in brackets)")
for C, res, relu in [(64, False, True), (256, True, True), (2048, True, True), (512, False, False)]:
    torch.manual_seed(C)
    bn = torch.nn.BatchNorm2d(C).to(dev)
    torch.nn.init.uniform_(bn.weight, 0.5, 1.5)
    torch.nn.init.uniform_(bn.bias, -0.5, 0.5)
    bn32 = torch.nn.BatchNorm2d(C).to(dev)
    bn32.load_state_dict(bn.state_dict())
    bn = bn.to(torch.bfloat16)
    bnt = copy.deepcopy(bn)
    H = 7 if C >= 1024 else 14
    x = (torch.randn(16, C, H, H, device=dev) * 2 + 0.5).to(torch.bfloat16).to(memory_format=torch.channels_last)
    r = torch.randn_like(x) if res else None
    xs = [x.clone().requires_grad_() for _ in range(2)]
    rs = [r.clone().requires_grad_() if res else None for _ in range(2)]
    y = bn_act(xs[0], bn, rs[0], relu)
    g = torch.randn_like(y)
    y.backward(g)
    with reference_ops():  # torch bf16
        yt = bnt(xs[1])
        if res:
            yt = yt + rs[1]
        if relu:
            yt = torch.relu(yt)
        yt.backward(g)
    x32 = x.detach().float().requires_grad_()
    r32 = r.detach().float().requires_grad_() if res else None
    y32 = bn32(x32)
    if res:
        y32 = y32 + r32
    if relu:
        y32 = torch.relu(y32)
    y32.backward(g.float())
    out = [f"C={C} res={res} relu={relu}:"]
    pairs = [("y", y, yt, y32), ("dx", xs[0].grad, xs[1].grad, x32.grad)]
    if res:
        pairs.append(("dres", rs[0].grad, rs[1].grad, r32.grad))
    pairs += [("dgamma", bn.weight.grad, bnt.weight.grad, bn32.weight.grad),
              ("dbeta", bn.bias.grad, bnt.bias.grad, bn32.bias.grad),
              ("run_mean", bn.running_mean, bnt.running_mean, bn32.running_mean),
              ("run_var", bn.running_var, bnt.running_var, bn32.running_var)]
    for n, a, t, ref in pairs:
        out.append(f"{n} {rel(a, ref):.4f} [{rel(t, ref):.4f}]")
    print("  ".join(out), flush=True)

print("== ResNet bottleneck oracle: worst e_nat / (e_t) per path and seed")
for bnm in ("fused", "torch"):
    for cm in ("gemm", "conv"):
        config.update(resnet_bn=bnm, resnet_conv1x1=cm)
        for seed in (6, 7, 8):
            torch.manual_seed(seed)
            m = resnet_tiny().to(dev)
            for mod in m.modules():
                if isinstance(mod, torch.nn.BatchNorm2d):
                    torch.nn.init.uniform_(mod.weight, 0.5, 1.5)
                    torch.nn.init.uniform_(mod.bias, -0.1, 0.1)
            m = m.to(torch.bfloat16).to(memory_format=torch.channels_last)
            x = torch.randn(16, 3, 32, 32, device=dev)
            yl = torch.randint(0, 10, (16,), device=dev)

            def loss_fn(mm):
                dt = next(mm.parameters()).dtype
                return mm(x.to(dt).to(memory_format=torch.channels_last), yl)

            oracle = copy.deepcopy(m).float()
            loss = loss_fn(m)
            loss.backward()
            gn = {n: p.grad.float().clone() for n, p in m.named_parameters()}
            m.zero_grad(set_to_none=True)
            with reference_ops():
                loss_fn(m).backward()
                loss_fn(oracle).backward()
            errs = []
            for n, po in oracle.named_parameters():
                ref = po.grad.float()
                den = ref.norm().item()
                if den == 0:
                    continue
                e_nat = (gn[n] - ref).norm().item() / den
                e_t = (m.get_parameter(n).grad.float() - ref).norm().item() / den
                errs.append((e_nat / (e_t + 1e-3), n, round(e_nat, 4), round(e_t, 4)))
            errs.sort(reverse=True)
            fail = [e for e in errs if e[2] > max(0.06, 1.25 * e[3] + 2e-3)]
            print(f"bn={bnm} conv1x1={cm} seed={seed}: worst {errs[:3]}  fails {len(fail)}", flush=True)
