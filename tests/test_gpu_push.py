"""Memory-pressure push between two server cores (adlb.c:509-556, 2109-2362).

Two adlbsrv handler sets on one GPU (server ranks 4 and 5 of 4 apps + 2
servers) exchange the SS_PUSH_* messages by hand: the pusher's loop-top
choice, the pushee's accept / decline, SS_PUSH_HDR + SS_PUSH_WORK with the
payload, the put-side match of a Reserve parked at the pushee, SS_PUSH_DEL
when a Reserve pinned the unit meanwhile, and SS_MOVING_TARGETED_WORK for a
targeted unit (the home server's tq then points at the new server, whose
SS_RFR serves the target rank).  The queue operations underneath are pinned
against the reference's xq.c by tests/golden/t17_push.npz
(test_gpu_parity.py::test_golden).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TYPES = [11, 22, 33, 44]
A_RANKS, PUSHER, PUSHEE = 4, 4, 5
T_RESERVE_RESP, T_RFR, T_RFR_RESP = 1008, 1018, 1019
T_QUERY, T_QRESP, T_HDR, T_WORK, T_DEL, T_MOVING = 1021, 1022, 1023, 1024, 1025, 1029


def hdr(wtype, prio, target=-1, length=600, home=PUSHER):
    return [wtype, prio, 0, target, length, home, 0, 0, -1, -1, 0, 0]


def req(*types):
    return [1, *types] + [-2] * (16 - len(types))


def ints(b):
    return np.frombuffer(b, np.int32)


def dbls(b):
    return np.frombuffer(b, np.float64)


def only(replies, tag):
    got = [r for r in replies if r[1] == tag]
    assert len(got) == 1, replies
    return got[0]


@pytest.fixture
def cores():
    from adlb_amd.core import Core
    # the pusher holds little (threshold 0.95 * 2000 B); the pushee has room
    with Core(TYPES, A_RANKS, 2, PUSHER, max_malloc=2000, device=0) as a, \
            Core(TYPES, A_RANKS, 2, PUSHEE, max_malloc=1e9, device=0) as b:
        yield a, b


def push_round(a, b, park=None):
    """query -> (optional Reserves parked at the pushee) -> resp -> hdr/work or del"""
    sent, q = a.push_tick()
    assert sent == 1
    dest, tag, qb = only(q, T_QUERY)
    assert dest == PUSHEE
    r = b.push_query(PUSHER, dbls(qb))
    _, _, rb = only(r, T_QRESP)
    if park is not None:
        park()
    out = a.push_query_resp(PUSHEE, dbls(rb))
    return dbls(qb), dbls(rb), out


def test_push_moves_unit_and_serves_parked_reserve(cores):
    a, b = cores
    payloads = [bytes([i]) * 600 for i in range(3)]
    for i, (t, p) in enumerate([(11, 7), (22, 5), (33, 9)]):
        a.put(0, hdr(t, p), payloads[i])
    # 3 x (96 + 600) B > 0.95 x 2000 B: the next loop-top check pushes
    parked = []

    def park():  # a Reserve for type 11 parks at the pushee: the held unit is not available yet
        parked.extend(b.reserve_batch([1], [req(11)]))
    q, r, out = push_round(a, b, park)
    # the query carries the first unpinned unit (wq_find_unpinned: seq 1) and its fields
    assert q[0] == 11 and q[1] == 7 and q[2] == 600 and q[5] == -1 and q[7] == 1
    assert r[0] == PUSHEE and r[2] == 1 and r[3] == 1  # accepted as the pushee's wqseqno 1
    assert parked == []
    d_hdr, d_work = only(out, T_HDR), only(out, T_WORK)
    assert d_hdr[0] == PUSHEE and ints(d_hdr[2])[0] == 1 and d_work[2] == payloads[0]
    assert b.push_len(1) == 600
    served = b.push_hdr(PUSHER, ints(d_hdr[2]), d_work[2])
    dest, _, rr = only(served, T_RESERVE_RESP)
    v = ints(rr)
    assert dest == 1 and list(v[:7]) == [1, 11, 7, 600, 0, 1, PUSHEE]
    got = b.get_batch([1], [1])
    assert got[-1][2] == payloads[0]
    assert a.info_get(3) == 1 and b.info_get(4) == 1  # ADLB_INFO_NPUSHED_FROM_HERE / _TO_HERE
    # below the threshold now: no further push
    assert a.push_tick()[0] == 0


def test_push_del_when_reserved_meanwhile(cores):
    a, b = cores
    for t in (11, 22, 33):
        a.put(0, hdr(t, 3), b"x" * 600)

    def pin_at_pusher():  # a Reserve at the pusher takes the queried unit before the answer
        r = a.reserve_batch([2], [req(11)])
        assert ints(only(r, T_RESERVE_RESP)[2])[5] == 1
    _, r, out = push_round(a, b, pin_at_pusher)
    d = only(out, T_DEL)
    assert d[0] == PUSHEE and ints(d[2])[0] == int(r[3])
    b.push_del(PUSHER, ints(d[2]))
    assert ints(b.info_num(0, 11)[0][2])[2] == 0  # the held unit is gone
    assert a.info_get(3) == 0 and b.info_get(4) == 0


def test_push_declined_when_pushee_full():
    from adlb_amd.core import Core
    with Core(TYPES, A_RANKS, 2, PUSHER, max_malloc=2000, device=0) as a, \
            Core(TYPES, A_RANKS, 2, PUSHEE, max_malloc=500, device=0) as b:
        for t in (11, 22, 33):
            a.put(0, hdr(t, 3), b"y" * 600)
        _, r, out = push_round(a, b)
        assert r[0] == -1 and out == []  # curr + len >= 0.95 max_malloc at the pushee (adlb.c:2122)
        assert a.info_get(3) == 0


def test_push_targeted_unit_moves_home_tq(cores):
    a, b = cores
    # seq 1 pinned by a Reserve, so the first unpinned unit is the targeted one (seq 2, rank 2)
    a.put(0, hdr(22, 4), b"p" * 600)
    a.put(0, hdr(33, 6, target=2), b"t" * 600)
    a.put(0, hdr(44, 1), b"q" * 600)
    a.reserve_batch([3], [req(22)])

    def park_target():  # the target rank parks at its home server once the unit has left
        pass
    q, r, out = push_round(a, b, park_target)
    assert q[0] == 33 and q[5] == 2 and q[6] == PUSHER
    assert a.reserve_batch([2], [req(33)]) == []  # parked at the pusher: no unit left for rank 2
    moved = b.push_hdr(PUSHER, ints(only(out, T_HDR)[2]), only(out, T_WORK)[2])
    dest, _, mb = only(moved, T_MOVING)
    assert dest == PUSHER and list(ints(mb)[:4]) == [2, 33, PUSHER, PUSHEE]
    # the home server's tq now points at the pushee: its check_remote sends rank 2's SS_RFR there
    rfr = a.moving_targeted(PUSHEE, ints(mb))
    dest, _, rb = only(rfr, T_RFR)
    assert dest == PUSHEE and list(ints(rb)[:3]) == [1, 2, 33]
    resp = b.rfr(PUSHER, ints(rb))
    _, _, sb = only(resp, T_RFR_RESP)
    s = ints(sb)
    assert s[0] == 1 and s[3] == 33 and s[8] == 2  # the targeted unit, prev_target 2
    done = a.rfr_resp(PUSHEE, s)
    dest, _, tb = only(done, T_RESERVE_RESP)
    assert dest == 2 and ints(tb)[1] == 33 and ints(tb)[6] == PUSHEE
