"""Join records that trail their ticket (VERDICT r5 weak #8 root cause).

A TCPStore ``set`` is not acknowledged: the client returns before the server applies it, so a
``check`` on another connection can be served first. The store-auth flake of round 5 was that race in
the test; the same race in the code lost joiners: ``join()`` takes its ticket with an (acknowledged)
``add`` on ``njoin`` and then posts ``join/<seq>`` with a ``set``, and a member that counted the
ticket while the record was still in flight recorded ``njoin`` in the next generation without the
joiner -- who then waited for an admission that never came. Reference analog: the ``join`` verb
(/root/reference/server.py:104-124), which has no ordering to get wrong.
"""
import datetime
import time

import torch.distributed as dist

from distributedvolunteercomputing_amd.parallel.elastic import ElasticMembership, _P


def _store():
    srv = dist.TCPStore("127.0.0.1", 0, None, True, timeout=datetime.timedelta(seconds=10))
    return srv


def test_set_is_not_acknowledged_but_add_orders_it():
    srv = _store()
    a = dist.TCPStore("127.0.0.1", srv.port, None, False, timeout=datetime.timedelta(seconds=10))
    big = "x" * (4 << 20)
    for i in range(8):
        a.set(f"k{i}", big)
        a.add("seq", 1)  # acknowledged, same connection: the set before it has been applied
        assert srv.check([f"k{i}"])


def test_pending_joiners_stop_at_a_ticket_without_its_record():
    srv = _store()
    m = ElasticMembership(srv, 0, lease_s=0.5)
    m.joins_seen = 0
    srv.add(f"{_P}njoin", 3)
    srv.set(f"{_P}join/1", "7")
    srv.set(f"{_P}join/3", "9")
    srv.add(f"{_P}sync", 1)
    # ticket 2's record has not arrived: only the joiner of ticket 1 is admitted, and the round's
    # outcome records njoin = 1, so ticket 2 stays pending instead of being consumed
    assert m._pending_joiners(3) == ([7], 1)
    srv.set(f"{_P}join/2", "8")
    srv.add(f"{_P}sync", 1)
    assert m._pending_joiners(3) == ([7, 8, 9], 3)


def test_a_ticket_whose_record_never_comes_is_skipped_after_the_lease():
    srv = _store()
    m = ElasticMembership(srv, 0, lease_s=0.2)
    srv.add(f"{_P}njoin", 2)
    srv.set(f"{_P}join/2", "5")
    srv.add(f"{_P}sync", 1)
    assert m._pending_joiners(2) == ([], 0)  # ticket 1's joiner died between its add and its set
    time.sleep(0.3)
    assert m._pending_joiners(2) == ([5], 2)


def test_round_with_a_trailing_record_defers_the_joiner_instead_of_consuming_its_ticket():
    srv = _store()
    member = ElasticMembership(srv, 0, lease_s=5.0, liveness=False)
    member.bootstrap([0])
    try:
        srv.add(f"{_P}njoin", 1)  # the joiner's ticket; its record is still in flight
        g = member.gen
        grp, changed, newcomers = member._round("1", recovery=False)
        assert srv.get(f"{_P}out/{g}/1").decode() == "same" and not changed
        assert member.joins_seen == 0  # the ticket was not consumed without its joiner
        srv.set(f"{_P}join/1", "4")
        srv.add(f"{_P}sync", 1)
        assert member._pending_joiners(1) == ([4], 1)  # the next round admits it
    finally:
        member.stop_heartbeat()
