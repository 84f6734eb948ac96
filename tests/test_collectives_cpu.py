"""All-reduce algorithms over gloo peer groups (CPU, multi-process)."""
import pytest
import torch

from tests import _mp


def _allreduce_worker(rank, world, port, algo, n):
    from distributedvolunteercomputing_amd.parallel.collectives import allreduce_sum_
    from distributedvolunteercomputing_amd.parallel.peer_group import PeerGroup

    store = _mp.make_store(rank, world, port)
    g = PeerGroup(store, rank, world, "gloo")
    torch.manual_seed(rank)
    t = torch.randn(n)
    ref = torch.zeros(n)
    for r in range(world):
        torch.manual_seed(r)
        ref += torch.randn(n)
    allreduce_sum_(t, g, algo)
    err = (t - ref).abs().max().item()
    g.barrier()
    return err


@pytest.mark.parametrize("algo", ["rccl", "rs_ag", "butterfly", "ring"])
@pytest.mark.parametrize("world", [2, 3, 4])
def test_allreduce_algorithms(algo, world):
    res = _mp.run(_allreduce_worker, world, algo, 1000)
    assert all(e < 1e-4 for e in res.values()), res


def test_butterfly_five_peers_odd_length():
    res = _mp.run(_allreduce_worker, 5, "butterfly", 777)
    assert all(e < 1e-4 for e in res.values()), res
