"""The cross-shard steal round on CPU.

The merge (adlbq_steal_merge, host code in libadlbq.so -- no GPU needed) over
numpy models of the shards' exports must settle exactly the Reserves the
serialised SS_RFR / SS_RFR_RESP exchanges settle on the oracle shards
(oracle.serial_steal_round: adlb.c:1280-1308, 1802-1933, 3487-3534), with the
same units and the same TA_RESERVE_RESP records; small k (several rounds)
gives the same result; the all-gather version over gloo (world size 2) equals
the in-process one.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle
from adlb_amd import shards
from adlb_amd._lib import AdlbqError
from steal_case import build_case, list_shards, rounds

if not oracle.available("own"):
    oracle.build()


@pytest.mark.parametrize("S,seed", [(2, 1), (3, 2), (5, 3)])
def test_merge_equals_serial_round(S, seed):
    ws, orcs, resps = build_case(S, n_units=600, R=96, seed=seed)
    ls = list_shards(ws, orcs, resps)
    nreq = sum(x.rq.shape[0] for x in ls)
    assert nreq > 0
    got, nd, settled, _ = shards.steal_round_local(ls, k=4096)
    assert nd == nreq
    exp = oracle.serial_steal_round(orcs, ws[0].num_app_ranks)
    assert exp.shape[0] > 0 and settled == exp.shape[0]
    np.testing.assert_array_equal(got, exp)
    # every shard's rq lost exactly the settled entries
    for s, x in enumerate(ls):
        np.testing.assert_array_equal(x.rq[:, 0], orcs[s].rq_list()[:, 0])


@pytest.mark.parametrize("k", [1, 2, 7])
def test_small_k_rounds_equal_serial_round(k):
    ws, orcs, resps = build_case(3, n_units=500, R=128, seed=11, prio_hi=8)
    ls = list_shards(ws, orcs, resps)
    got = rounds(lambda: shards.steal_round_local(ls, k=k))
    exp = oracle.serial_steal_round(orcs, ws[0].num_app_ranks)
    np.testing.assert_array_equal(got, exp)


def test_wildcard_and_ties_pick_lowest_shard():
    """Equal head priorities on every donor: the lowest shard index wins
    (strict > from LOWEST, adlb.c:3510-3529), for typed and wildcard requests."""
    ut = np.arange(2, dtype=np.int32)
    S, T, k = 3, 2, 4
    recs = np.zeros((S, T, k, 8), np.int32)
    nrec = np.zeros((S, T), np.int32)
    navail = np.zeros((S, T), np.int64)
    for s in (1, 2):
        for t in range(T):
            recs[s, t, 0] = [50, 10 * s + t + 1, t, 8, 0, 0, -1, -1]
            nrec[s, t] = navail[s, t] = 1
    reqs = np.full((3, 19), -2, np.int32)
    reqs[:, 0] = 0
    reqs[:, 1] = [1, 2, 3]
    reqs[:, 2] = [5, 6, 7]
    reqs[0, 3] = 1          # type 1: shard 1
    reqs[1, 3] = -1         # wildcard: shard 1 (its remaining type 0)
    reqs[2, 3:5] = [1, 0]   # type 1: shard 2 (shard 1's is gone); unit = best of {0, 1} there: type 0, seq 21
    out, nd = shards.steal_merge(ut, k, recs, nrec, navail, reqs)
    assert nd == 3
    assert out.tolist() == [[1, 1, 0], [1, 0, 0], [2, 0, 0]]


def test_stops_at_unknown_and_no_donor():
    ut = np.arange(1, dtype=np.int32)
    recs = np.zeros((2, 1, 1, 8), np.int32)
    recs[1, 0, 0] = [9, 1, 0, 8, 0, 0, -1, -1]
    nrec = np.array([[0], [1]], np.int32)
    navail = np.array([[0], [5]], np.int64)       # shard 1 has more than it exported
    reqs = np.full((3, 19), -2, np.int32)
    reqs[:, 0], reqs[:, 1], reqs[:, 2], reqs[:, 3] = 0, [1, 2, 3], [4, 5, 6], 0
    out, nd = shards.steal_merge(ut, 1, recs, nrec, navail, reqs)
    assert nd == 1 and out.tolist() == [[1, 0, 0], [-1, -1, -1], [-1, -1, -1]]
    # a request on the only holder has no donor (own shard excluded)
    reqs[:, 0] = 1
    out, nd = shards.steal_merge(ut, 1, recs, nrec, navail, reqs)
    assert nd == 3 and (out == -1).all()


def test_merge_rejects_bad_input():
    ut = np.arange(1, dtype=np.int32)
    recs = np.zeros((2, 1, 1, 8), np.int32)
    nrec = np.zeros((2, 1), np.int32)
    navail = np.zeros((2, 1), np.int64)
    reqs = np.full((2, 19), -2, np.int32)
    reqs[:, 0], reqs[:, 1] = [1, 0], [1, 2]            # shard order broken
    with pytest.raises(AdlbqError):
        shards.steal_merge(ut, 1, recs, nrec, navail, reqs)
    reqs[:, 0] = 0
    with pytest.raises(AdlbqError):
        shards.steal_merge(ut, 1, recs, np.full((2, 1), 2, np.int32), navail, reqs)   # nrec > k


# ------------------------------------------------------------------ gloo world size 2
def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ws, orcs, resps = build_case(4, n_units=400, R=64, seed=21)
        ls = list_shards(ws, orcs, resps)
        mine = [x for x in ls if x.my_server_idx % world == rank]   # shards {rank, rank + 2}
        got = rounds(lambda: shards.steal_round(mine, k=3))
        q.put((rank, got.tolist(), [x.rq[:, 0].tolist() for x in mine]))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def test_steal_round_allgather_gloo():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r = q.get(timeout=120)
        got[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ws, orcs, resps = build_case(4, n_units=400, R=64, seed=21)
    exp = oracle.serial_steal_round(orcs, ws[0].num_app_ranks)
    assert exp.shape[0] > 0
    for r in range(world):
        g = np.asarray(got[r][1], np.int32).reshape(-1, 15)
        e = exp[exp[:, 0] % world == r]
        # each process returns its own shards' settlements, round by round
        np.testing.assert_array_equal(g[np.lexsort((g[:, 1], g[:, 0]))], e[np.lexsort((e[:, 1], e[:, 0]))])
        for s, left in zip([r, r + 2], got[r][2]):
            assert left == orcs[s].rq_list()[:, 0].tolist()


# ------------------------------------------------------------------ the bench's array restatement
def _array_shards(ws, resps, orcs):
    out = []
    for s, w in enumerate(ws):
        un = w.u_target < 0
        seq = np.arange(1, w.n_units + 1, dtype=np.int32)
        taken = np.zeros(w.n_units, bool)
        r = resps[s]
        taken[r[r[:, 0] == 1, 5] - 1] = True
        out.append({"type": w.u_type[un], "prio": w.u_prio[un], "seq": seq[un], "len": w.u_len[un],
                    "answer": w.u_answer[un], "avail": ~taken[un], "rq": orcs[s].rq_list()})
    return out


@pytest.mark.parametrize("S,seed,kw", [(2, 41, {}), (3, 43, {}), (4, 3, dict(p_remote=0.1, prio_hi=1024)),
                                       (3, 47, dict(prio_hi=4))])
def test_serial_steal_expect_matches_oracle(S, seed, kw):
    """exact_check.serial_steal_expect (the bench's config-3 round check, over
    sorted arrays) equals oracle.serial_steal_round (the RFR exchanges
    serialised over the restated linked lists) on the steal-round cases."""
    from exact_check import serial_steal_expect
    ws, orcs, resps = build_case(S, n_units=3000, R=512, seed=seed, **kw)
    sh = _array_shards(ws, resps, orcs)
    n = sum(x["rq"].shape[0] for x in sh)
    got = serial_steal_expect(ws[0].user_types, ws[0].num_app_ranks, sh, n)
    exp = oracle.serial_steal_round(orcs, ws[0].num_app_ranks)
    assert exp.shape[0] > 0
    np.testing.assert_array_equal(got, exp)
    # a decided prefix: the rows of the first requests only
    cut = sh[0]["rq"].shape[0] + 3
    part = serial_steal_expect(ws[0].user_types, ws[0].num_app_ranks, _array_shards(ws, resps, build_case(
        S, n_units=3000, R=512, seed=seed, **kw)[1]), cut)
    keep = (exp[:, 0] == 0) | ((exp[:, 0] == 1) & np.isin(exp[:, 1], sh[1]["rq"][:3, 0]))
    np.testing.assert_array_equal(part, exp[keep])
