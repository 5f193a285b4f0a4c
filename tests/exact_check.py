"""Size-independent exact check of a Reserve batch (test infrastructure).

Sequential FA_RESERVE handling (src/adlb.c:1199-1237 with xq.c:190-247) gives
request j the best available unit -- priority descending, then wqseqno
ascending -- first among units targeted at its rank, else among untargeted
units, restricted to its types.  Because every request ranks units by the same
key, an assignment equals that sequential result iff it is *stable*:

  for every request j and every type t it accepts, every unit of that pool
  (the rank's targeted pool, then the untargeted pool) that is better than
  what j received -- or every unit of the pool if j received nothing from it --
  was taken by an earlier request i < j.

(Induction on j: request 0 must get the pool maximum; request j gets the best
unit not taken by 0..j-1.)  This module checks that condition with sorting and
prefix maxima in O(N log N + R*T), so it runs at the 10M-unit BASELINE sizes
where replaying the reference's linked-list scans would take hours.
"""
from __future__ import annotations

import numpy as np

LOWEST = -999999999


def unit_keys(prio: np.ndarray, seq: np.ndarray) -> np.ndarray:
    """uint64 key, larger == better (prio desc, wqseqno asc)."""
    hi = (prio.astype(np.int64) + (1 << 31)).astype(np.uint64) << np.uint64(32)
    return hi | (np.uint64(0xFFFFFFFF) - seq.astype(np.uint64))


def check_batch(user_types, u_type, u_prio, u_target, u_seq, u_avail, r_rank, r_types, r_hang, resp,
                verbose: bool = False, u_len=None, u_answer=None, u_common=None, server_rank=None) -> dict:
    """Raise AssertionError with a description unless `resp` (R x 12) is the
    sequential result for the batch.  Units are given in any order with their
    wqseqno; u_avail marks units unpinned before the batch.  With u_len /
    u_answer / u_common (N x 3: common_len, common_server, common_seqno) /
    server_rank, the rest of every TA_RESERVE_RESP record is checked as well
    (adlb.c:1213-1224: len, answer_rank, server_rank, the common triple; -1 in
    words 10-11 of a request that did not park)."""
    ut = np.asarray(user_types)
    T = ut.size
    tmap = {int(v): i for i, v in enumerate(ut)}
    lut_vals, inv = np.unique(u_type, return_inverse=True)
    tidx = np.array([tmap[int(v)] for v in lut_vals], dtype=np.int64)[inv]
    N, R = u_type.size, r_rank.size
    resp = np.asarray(resp).reshape(R, 12)
    # request masks
    rt = np.asarray(r_types).reshape(R, 16)
    wild = (rt == -1).any(axis=1)
    acc = np.zeros((R, T), dtype=bool)
    for t in range(T):
        acc[:, t] = (rt == ut[t]).any(axis=1) | wild
    matched = resp[:, 0] == 1
    # owners
    seq_max = int(u_seq.max()) + 1 if N else 1
    slot_of_seq = np.full(seq_max, -1, dtype=np.int64)
    slot_of_seq[u_seq] = np.arange(N)
    mseq = resp[matched, 5]
    assert (mseq > 0).all() and (mseq < seq_max).all(), "matched wqseqno out of range"
    mslot = slot_of_seq[mseq]
    assert (mslot >= 0).all(), "matched wqseqno unknown"
    assert np.unique(mslot).size == mslot.size, "a unit was given to two requests"
    owner = np.full(N, R, dtype=np.int64)
    jm = np.nonzero(matched)[0]
    owner[mslot] = jm
    # response fields and basic eligibility
    assert u_avail[mslot].all(), "matched a unit pinned before the batch"
    assert (u_type[mslot] == resp[matched, 1]).all(), "type field"
    assert (u_prio[mslot] == resp[matched, 2]).all(), "prio field"
    assert (u_prio[mslot] > LOWEST).all(), "matched a LOWEST_PRIO unit"
    assert acc[jm, tidx[mslot]].all(), "matched a type the request did not ask for"
    tg = u_target[mslot]
    assert ((tg < 0) | (tg == r_rank[jm])).all(), "matched another rank's targeted unit"
    unm = ~matched
    assert ((resp[unm, 0] == 0) == (r_hang[unm] != 0)).all(), "park vs NO_CURR_WORK"
    assert (resp[unm & (r_hang == 0), 0] == -2).all()
    if u_len is not None:
        assert (np.asarray(u_len)[mslot] == resp[matched, 3]).all(), "len field"
    if u_answer is not None:
        assert (np.asarray(u_answer)[mslot] == resp[matched, 4]).all(), "answer_rank field"
    if server_rank is not None:
        assert (resp[matched, 6] == server_rank).all(), "server_rank field"
    if u_common is not None:
        assert (np.asarray(u_common).reshape(-1, 3)[mslot] == resp[matched, 7:10]).all(), "common fields"
    if u_len is not None or u_common is not None:
        parked = resp[:, 0] == 0
        assert (resp[~parked, 10:12] == -1).all(), "words 10-11 of a request that did not park"
        assert (resp[unm & (r_hang == 0), 1:10] == 0).all(), "NO_CURR_WORK record"

    elig = u_avail & (u_prio > LOWEST)
    key = unit_keys(u_prio, u_seq)
    order = np.lexsort((np.uint64(0xFFFFFFFFFFFFFFFF) - key,))  # ascending of inverted == descending key
    grank = np.empty(N, dtype=np.int64)
    grank[order] = np.arange(N)               # 0 == best unit overall
    g_req = np.full(R, N, dtype=np.int64)      # global rank of what j got (N == nothing)
    g_req[jm] = grank[mslot]
    got_targeted = np.zeros(R, dtype=bool)
    got_targeted[jm] = u_target[mslot] >= 0
    checks = 0
    for t in range(T):
        need = acc[:, t]
        if not need.any():
            continue
        # --- untargeted pool of type t
        pool = elig & (tidx == t) & (u_target < 0)
        pr = np.sort(grank[pool])
        pown = owner[pool][np.argsort(grank[pool])]
        pmax = np.maximum.accumulate(pown) if pown.size else pown
        js = np.nonzero(need & ~got_targeted)[0]
        cnt = np.searchsorted(pr, g_req[js], side="left")
        bad = (cnt > 0) & (pmax[np.maximum(cnt - 1, 0)] >= js) if pr.size else np.zeros(js.size, bool)
        assert not bad.any(), f"untargeted type {ut[t]}: request {js[bad][0]} skipped a better free unit"
        checks += js.size
        # --- targeted pools (rank, t)
        tpool = elig & (tidx == t) & (u_target >= 0)
        if tpool.any():
            comp = u_target[tpool].astype(np.int64) * (1 << 32) + grank[tpool]
            o = np.argsort(comp)
            comp = comp[o]
            town = owner[tpool][o]
            tgt_sorted = u_target[tpool][o]
            # prefix max restarted per segment
            seg_start = np.r_[0, np.nonzero(np.diff(tgt_sorted))[0] + 1]
            seg_id = np.repeat(np.arange(seg_start.size), np.diff(np.r_[seg_start, tgt_sorted.size]))
            big = town + seg_id.astype(np.int64) * (R + 1) * 4
            tmax = np.maximum.accumulate(big) - seg_id.astype(np.int64) * (R + 1) * 4
            js = np.nonzero(need)[0]
            lo = np.searchsorted(comp, r_rank[js].astype(np.int64) * (1 << 32), side="left")
            # requests that got an untargeted unit (or nothing) must have found the pool empty
            lim = np.where(got_targeted[js], g_req[js], 1 << 32)
            hi = np.searchsorted(comp, r_rank[js].astype(np.int64) * (1 << 32) + lim, side="left")
            nz = hi > lo
            bad = nz & (tmax[np.maximum(hi - 1, 0)] >= js)
            assert not bad.any(), f"targeted type {ut[t]}: request {js[bad][0]} skipped a better free unit"
            checks += js.size
    return {"matched": int(matched.sum()), "checks": checks}


def serial_steal_expect(user_types, num_app_ranks: int, shards, n_decided: int) -> np.ndarray:
    """The steal round the cross-shard merge replaces, restated over sorted
    arrays (size-independent; the oracle's serial_steal_round does the same
    over linked lists, too slow at config 3's 1.5M units per shard).

    shards: per shard index s, a dict with the shard's untargeted units
    (type, prio, seq, len, answer: arrays; avail: bool, unpinned before the
    round) and its parked Reserves in rqseqno order (rq: (m, 18) {rqseqno,
    rank, types[16]}).  The parked Reserves of shard 0, 1, ... in rqseqno
    order, the first n_decided of them, each pick a donor on the current
    qmstat rows (find_cand_rank_with_worktype, adlb.c:3487-3534: the first
    type in request order with a server != self whose row has qlen > 0 and the
    highest type_hi_prio, lowest index on ties); the donor answers SS_RFR with
    its best unit over the request's types (wq_find_hi_prio, xq.c:190-217;
    adlb.c:1817-1846), its row changes, and the requester replies
    TA_RESERVE_RESP with the donor's world rank (adlb.c:1884-1898).
    Returns (n, 15) {shard, rqseqno, rank, TA_RESERVE_RESP[12]} per steal."""
    ut = [int(x) for x in np.asarray(user_types)]
    T, S = len(ut), len(shards)
    lists, head, qlen = [], np.zeros((S, T), np.int64), np.zeros(S, np.int64)
    for s, sh in enumerate(shards):
        ok = np.asarray(sh["avail"], bool)
        qlen[s] = int(ok.sum())
        el = ok & (np.asarray(sh["prio"]) > LOWEST)
        per = []
        for t in range(T):
            idx = np.nonzero(el & (np.asarray(sh["type"]) == ut[t]))[0]
            per.append(idx[np.lexsort((np.asarray(sh["seq"])[idx], -np.asarray(sh["prio"])[idx].astype(np.int64)))])
        lists.append(per)

    def hi(s, t):
        L = lists[s][t]
        return int(shards[s]["prio"][L[head[s, t]]]) if head[s, t] < L.size else LOWEST

    out, done = [], 0
    for s, sh in enumerate(shards):
        for e in np.asarray(sh["rq"]).reshape(-1, 18):
            if done >= n_decided:
                break
            done += 1
            rqseqno, rank, types = int(e[0]), int(e[1]), [int(v) for v in e[2:]]
            d = -1
            for v in types:
                if v < -1:
                    break
                best, bh = -1, LOWEST
                for j in range(S):
                    if j == s or qlen[j] <= 0:
                        continue
                    for t in (range(T) if v == -1 else ([ut.index(v)] if v in ut else [])):
                        x = hi(j, t)
                        if x > bh:
                            bh, best = x, j
                if best >= 0:
                    d = best
                    break
            if d < 0:
                continue
            wild = any(v == -1 for v in types)   # xq.c:199-207 tests all 16 entries
            cand = range(T) if wild else sorted({ut.index(v) for v in types if v in ut})
            bt, bk = -1, None
            for t in cand:
                L = lists[d][t]
                if head[d, t] < L.size:
                    u = L[head[d, t]]
                    k = (-int(shards[d]["prio"][u]), int(shards[d]["seq"][u]))
                    if bk is None or k < bk:
                        bt, bk = t, k
            assert bt >= 0, "a donor chosen on a fresh table must have a unit"
            u = lists[d][bt][head[d, bt]]
            head[d, bt] += 1
            qlen[d] -= 1
            D = shards[d]
            out.append([s, rqseqno, rank, 1, int(D["type"][u]), int(D["prio"][u]), int(D["len"][u]),
                        int(D["answer"][u]), int(D["seq"][u]), num_app_ranks + d, 0, -1, -1, -1, -1])
    return np.asarray(out, dtype=np.int32).reshape(-1, 15)
