"""Flat parameter storage (parallel/flat_params.py): channels-last convolution weights keep their
memory format in the flat buffer (no layout copy per step for NHWC convolution kernels), and a
checkpoint records it (utils/checkpoint.py refuses a layout with other memory formats)."""
import pytest
import torch

from distributedvolunteercomputing_amd.models.resnet import resnet_tiny
from distributedvolunteercomputing_amd.parallel.flat_params import FlatParams, segment_view
from distributedvolunteercomputing_amd.utils import checkpoint


def test_channels_last_segments_keep_layout_and_values():
    torch.manual_seed(0)
    m = resnet_tiny().to(memory_format=torch.channels_last)
    ref = {n: p.detach().clone() for n, p in m.named_parameters()}
    f = FlatParams(m, dtype=torch.float32)
    cl = {s.name for s in f.segments if s.channels_last}
    # the 3x3 / 7x7 convolutions (1x1 kernels are plain-contiguous either way)
    assert cl and all(dict(m.named_parameters())[n].shape[-1] > 1 for n in cl)
    for n, p in m.named_parameters():
        assert torch.equal(p.detach(), ref[n]), n
        assert p.grad.stride() == p.stride(), n
        if n in cl:
            assert p.is_contiguous(memory_format=torch.channels_last) and not p.is_contiguous()
    # gradients written through autograd land in the flat buffer, in the segment's element order
    x = torch.randn(2, 3, 32, 32).to(memory_format=torch.channels_last)
    m(x, torch.tensor([1, 2])).backward()
    for s, p in zip(f.segments, f._params):
        assert p.grad.data_ptr() == f.grad[s.offset:].data_ptr()
        assert torch.equal(segment_view(f.grad, s), p.grad)
    views = f.state_dict_views(f.param)
    for n, p in m.named_parameters():
        assert torch.equal(views[n], p.detach())


def test_checkpoint_layout_checks_memory_format():
    m_cl = resnet_tiny().to(memory_format=torch.channels_last)
    m_std = resnet_tiny()
    f_cl, f_std = FlatParams(m_cl, dtype=torch.float32), FlatParams(m_std, dtype=torch.float32)

    class _M:  # the manifest part check_layout reads
        def __init__(self, flat):
            self.manifest = {"flat": checkpoint.layout_dict(flat)}

    checkpoint.ShardReader.check_layout(_M(f_cl), f_cl)
    with pytest.raises(ValueError, match="memory formats"):
        checkpoint.ShardReader.check_layout(_M(f_cl), f_std)
