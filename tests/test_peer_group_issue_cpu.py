"""A collective whose ISSUE fails because the watchdog aborted the communicator between the group's
check and the issue (seen in the 8-rank RCCL rehearsal: survivors crashed with a DistBackendError raised
by alltoall_base itself) is a PeerFailure under a watch -- the round is redone on the survivors -- and the
original error without one (parallel/peer_group.py PeerGroup._issue)."""
import threading

import pytest
import torch

from distributedvolunteercomputing_amd.parallel.peer_group import PeerFailure, PeerGroup


class _AbortedPG:
    def alltoall_base(self, *a, **k):
        raise RuntimeError("NCCL communicator was aborted on rank 3.")

    def allreduce(self, *a, **k):
        raise RuntimeError("NCCL communicator was aborted on rank 3.")


class _Watch:
    pid = 0

    def __init__(self):
        self.reasons = []

    def tripped(self):
        return False

    def declare_abort(self, why):
        self.reasons.append(why)

    def abort_reason(self):
        return self.reasons[-1] if self.reasons else ""


def _group(watch):
    g = PeerGroup.__new__(PeerGroup)
    g._pending = g._bg = None
    g.generation, g.size, g.rank, g.members = 3, 4, 0, [0, 1, 2, 3]
    g.backend, g.device, g.watch, g.aborted = "gloo", None, watch, False
    g._abort_lock = threading.Lock()
    g.fault_hook, g.poll_s = None, 1e-4
    g.pg = _AbortedPG()
    return g


def test_issue_failure_under_watch_is_peer_failure():
    w = _Watch()
    g = _group(w)
    t = torch.zeros(8)
    with pytest.raises(PeerFailure):
        g.alltoall_(t, t.clone(), [2, 2, 2, 2], [2, 2, 2, 2])
    assert g.aborted and g.pg is None and "alltoall issue failed" in w.reasons[-1]
    with pytest.raises(PeerFailure):  # torn down: the next collective fails the same way
        g.allreduce_(t)


def test_issue_failure_without_watch_raises_the_error():
    g = _group(None)
    with pytest.raises(RuntimeError, match="aborted"):
        g.allreduce_(torch.zeros(4))


class _BuggyPG:
    def allreduce(self, *a, **k):
        raise ValueError("split sizes do not match the tensor")

    def alltoall_base(self, *a, **k):
        raise RuntimeError("Split sizes doesn't match total dim 0 size")


def test_caller_bug_under_watch_stays_a_crash():
    """only transport / abort failures become a PeerFailure (a redone round); a caller's
    shape or split mistake is re-raised unchanged and declares no abort."""
    w = _Watch()
    g = _group(w)
    g.pg = _BuggyPG()
    with pytest.raises(ValueError, match="split sizes"):
        g.allreduce_(torch.zeros(4))
    t = torch.zeros(8)
    with pytest.raises(RuntimeError, match="Split sizes"):
        g.alltoall_(t, t.clone(), [2, 2, 2, 2], [2, 2, 2, 2])
    assert w.reasons == [] and not g.aborted and g.pg is not None
