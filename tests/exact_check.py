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
                verbose: bool = False) -> dict:
    """Raise AssertionError with a description unless `resp` (R x 12) is the
    sequential result for the batch.  Units are given in any order with their
    wqseqno; u_avail marks units unpinned before the batch."""
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
