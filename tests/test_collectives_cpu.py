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


ALGOS = ["rccl", "rs_ag", "butterfly", "ring", "direct"]


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("world", [2, 3, 4])
def test_allreduce_algorithms(algo, world):
    res = _mp.run(_allreduce_worker, world, algo, 1000)
    assert all(e < 1e-4 for e in res.values()), res


def _all_algos_worker(rank, world, port, n, dtype):
    from distributedvolunteercomputing_amd.parallel.collectives import allreduce_sum_
    from distributedvolunteercomputing_amd.parallel.peer_group import PeerGroup

    store = _mp.make_store(rank, world, port)
    g = PeerGroup(store, rank, world, "gloo")
    ref = sum(torch.randn(n, generator=torch.Generator().manual_seed(r)) for r in range(world))
    out = {}
    for algo in ALGOS:
        t = torch.randn(n, generator=torch.Generator().manual_seed(rank)).to(dtype)
        allreduce_sum_(t, g, algo)
        out[algo] = (t.float() - ref).abs().max().item() / ref.abs().max().item()
    g.barrier()
    return out


@pytest.mark.parametrize("world", [5, 8])
def test_every_algorithm_at_larger_worlds(world):
    """P = 8 (one volunteer per MI355X of a node) and a non-power-of-two P, every algorithm."""
    res = _mp.run(_all_algos_worker, world, 4096 + 64, torch.float32, timeout=180)
    for r, errs in res.items():
        assert all(e < 1e-5 for e in errs.values()), (r, errs)


def test_direct_bf16_four_peers():
    res = _mp.run(_all_algos_worker, 4, 2048, torch.bfloat16)
    for r, errs in res.items():
        assert errs["direct"] < 2e-2, (r, errs)


def test_butterfly_five_peers_odd_length():
    res = _mp.run(_allreduce_worker, 5, "butterfly", 777)
    assert all(e < 1e-4 for e in res.values()), res
