"""A worker asked to send a result it no longer holds sends a TAGGED placeholder (the pair FIFO needs
a buffer of the announced shape); the requester recognises the tag and re-submits the chunk instead
of delivering black frames. Reference: a lost chunk is never recovered at all
(/root/reference/worker.py:214-239)."""
import torch

from distributedvolunteercomputing_amd.control.peer import _is_placeholder, _placeholder


def test_placeholder_is_recognised_and_real_chunks_are_not():
    shape = (100, 225, 400, 3)
    ph = _placeholder(shape)
    assert tuple(ph.shape) == shape and ph.dtype == torch.uint8
    assert _is_placeholder(ph)
    assert not _is_placeholder(torch.zeros(shape, dtype=torch.uint8))  # an all-black real chunk
    g = torch.Generator().manual_seed(0)
    assert not _is_placeholder(torch.randint(0, 256, shape, dtype=torch.uint8, generator=g))
    assert not _is_placeholder(_placeholder((8,)))  # too small to carry the tag: never a match
