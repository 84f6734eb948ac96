"""ops/linear.py subsample_tap: the stride-2 shortcut convolution's input and the gradient join of a
projection-shortcut ResNet block (conv1 deposits its input gradient; the tap adds the strided
quarter into it instead of autograd's zero-filled slice gradient + full-size add)."""
import torch

from distributedvolunteercomputing_amd.ops.linear import GradJoin, subsample_tap


def _x():
    torch.manual_seed(0)
    return torch.randn(2, 5, 6, 8).to(memory_format=torch.channels_last).requires_grad_()


def test_forward_is_the_strided_nhwc_subsample():
    x = _x()
    xs = subsample_tap(x, GradJoin(), 2)
    assert xs.is_contiguous() and xs.shape == (2, 3, 4, 5)
    assert torch.equal(xs, x.permute(0, 2, 3, 1)[:, ::2, ::2, :])


def test_backward_adds_into_the_deposited_gradient():
    x = _x()
    j = GradJoin()
    xs = subsample_tap(x, j, 2)
    dep = torch.randn(2 * 6 * 8, 5)
    j.pending = dep.clone()  # what conv1's backward leaves (ops/linear.py _Linear, deposit=True)
    g = torch.randn_like(xs)
    xs.backward(g)
    want = dep.view(2, 6, 8, 5).clone()
    want[:, ::2, ::2, :] += g
    assert torch.equal(x.grad, want.permute(0, 3, 1, 2))
    assert j.pending is None and not j.ran


def test_backward_without_a_deposit_is_the_plain_slice_gradient():
    x = _x()
    j = GradJoin()
    xs = subsample_tap(x, j, 2)
    g = torch.randn_like(xs)
    xs.backward(g)
    ref = x.detach().clone().requires_grad_()
    ref.permute(0, 2, 3, 1)[:, ::2, ::2, :].contiguous().backward(g)
    assert torch.equal(x.grad, ref.grad)
    assert j.ran  # conv1 (running later) then returns its own gradient to autograd
