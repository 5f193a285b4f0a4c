"""Parity of the HIP path (through the C ABI) with the oracle and the reference.

* golden fixtures (expected streams generated from the reference's src/xq.c):
  the ABI replay must reproduce them bit for bit;
* fresh seeded traces at medium sizes: ABI replay == oracle replay;
* BASELINE sizes (10M-unit queue, 64K Reserves): the exact stability check of
  tests/exact_check.py (equivalent to sequential xq matching).
"""
import glob
import hashlib
import os
import sys

import numpy as np
import pytest

import oracle
from adlb_amd import replay, synth
from adlb_amd.server import Server
from exact_check import check_batch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))

pytestmark = pytest.mark.gpu
# server event streams (nq_*, mix_*: oracle/gen_nq.py) are replayed by test_gpu_server.py
GOLD = sorted(p for p in glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.npz"))
              if not os.path.basename(p).startswith(("nq_", "mix_")))


def run_abi(ut, cfg, trace, max_units=1 << 16, params=None, stats=None):
    with Server(ut, int(cfg[0]), int(cfg[1]), int(cfg[2]), max_units=max_units) as s:
        for k, v in (params or {}).items():
            s.set_param(k, v)
        out = replay.replay(s, trace)
        assert s.stat("sort_timeouts") == 0, "k_rank timed out waiting for an in-launch sort"
        if stats is not None:
            stats.update({k: s.stat(k) for k in ("chain_passes", "chain_recomputed", "chain_fallback",
                                                 "chain_timeouts", "spec_lists", "rank_fast", "keyrank",
                                                 "keyrank_failed")})
        return out


_ORACLE_MEMO = {}


def run_oracle(ut, cfg, trace):
    """The oracle's outputs for a trace, computed once per session per (types, cfg, trace):
    the variant tests replay the same seeded traces through several engine paths."""
    tr = np.ascontiguousarray(trace, dtype=np.int32)
    key = (tuple(int(x) for x in ut), tuple(int(x) for x in cfg), hashlib.sha1(tr.tobytes()).hexdigest())
    if key not in _ORACLE_MEMO:
        o = oracle.Oracle("own")
        o.init(ut, int(cfg[0]), int(cfg[1]), int(cfg[2]))
        _ORACLE_MEMO[key] = o.replay(tr)
    return _ORACLE_MEMO[key].copy()


def assert_same(got, exp):
    assert got.size == exp.size, (got.size, exp.size)
    bad = np.nonzero(got != exp)[0]
    assert bad.size == 0, f"first mismatch at output int {bad[0]}: got {got[bad[0]]} expected {exp[bad[0]]}"


# small open buckets and batches take the one-workgroup choice by default
# (k_reserve_small); "pipeline" turns it off so that the batch pipeline is
# checked on the same small cases
ENGINES = {"default": {}, "pipeline": {"small_pages": 0, "reserve_one": 0}}


@pytest.mark.parametrize("engine", sorted(ENGINES))
@pytest.mark.parametrize("path", GOLD, ids=[os.path.basename(p)[:-4] for p in GOLD])
def test_golden(gpu_available, path, engine):
    d = np.load(path, allow_pickle=False)
    assert_same(run_abi(d["user_types"], d["cfg"], d["trace"], params=ENGINES[engine]), d["expected"])


SMALL = {
    "s_c2_t4": lambda: synth.config2(n_units=16_000, n_reserves=1024, seed=601),
    "s_c2_t1_eq": lambda: synth.config2(n_units=3_000, n_types=1, n_reserves=1000, seed=602, equal_prio=True),
    "s_c2_exhaust": lambda: synth.config2(n_units=500, n_reserves=1000, seed=603, prio_hi=8),
    "s_c2_exhaust_nohang": lambda: synth.config2(n_units=500, n_reserves=1000, seed=604, hang=0),
    "s_c2_t8_extreme": lambda: synth.config2(n_units=8_000, n_types=8, n_reserves=1024, seed=605, wide_frac=0.1,
                                             wide_range=(-(1 << 31), (1 << 31) - 1)),
    "s_c2_t64": lambda: synth.config2(n_units=5_000, n_types=64, n_reserves=1024, seed=606, prio_hi=64),
    "s_c4_targeted": lambda: synth.config4(n_units=6_000, n_reserves=1024, n_ranks=64, seed=607, prio_hi=16),
    "s_c4_t8_tied": lambda: synth.config4(n_units=4_000, n_types=8, n_reserves=1024, n_ranks=32, seed=608, prio_hi=4),
    "s_r1": lambda: synth.config2(n_units=500, n_reserves=1, seed=609),
    # at most 256 Reserves: block minima over the units in registers instead of the sort
    "s_c2_r200_t8": lambda: synth.config2(n_units=12_000, n_types=8, n_reserves=200, seed=610, prio_hi=4),
    "s_c4_r256": lambda: synth.config4(n_units=9_000, n_reserves=256, n_ranks=32, seed=611, prio_hi=8),
    "s_c2_r256_exhaust": lambda: synth.config2(n_units=100, n_reserves=256, seed=612, prio_hi=3),
}


@pytest.mark.parametrize("engine", sorted(ENGINES))
@pytest.mark.parametrize("name", sorted(SMALL))
def test_small_queue_vs_oracle(gpu_available, name, engine):
    """Small open buckets (at most four pages) and batches (at most 1024): the
    one-workgroup choice and the batch pipeline both give the oracle's result."""
    w = SMALL[name]()
    tr = synth.workload_trace(w)
    cfg = (w.num_app_ranks, 1, 0)
    with Server(w.user_types, *cfg, max_units=w.n_units) as s:
        for k, v in ENGINES[engine].items():
            s.set_param(k, v)
        got = replay.replay(s, tr)
        used = s.stat("small_batches") + s.stat("one_batches")  # (a one-Reserve batch takes k_reserve_one)
        assert s.stat("bound_faults") == 0  # no choice outside the page list (DESIGN.md §9, round-5 fault)
    assert_same(got, run_oracle(w.user_types, cfg, tr))
    assert (used > 0) == (engine == "default"), used


@pytest.mark.parametrize("recycle", [1, 0])
def test_dead_pages_recycled_vs_oracle(gpu_available, recycle):
    """A long stream on a small queue: rounds of Puts, Reserve batches and Gets
    of every match leave whole pages dead; they leave the open bucket in the
    background (k_page_dead) and later Puts reuse them.  The results equal the
    oracle's with and without recycling, and the bucket stays small."""
    rng = np.random.default_rng(71)
    ut, A = [3, 5, 7], 256
    o = oracle.Oracle("own")
    o.init(ut, A, 1, 0)
    trace, exp = [], []

    def step(ev):
        ev = np.asarray(ev, dtype=np.int32).ravel()
        out = o.replay(ev)
        trace.append(ev)
        exp.append(out)
        return synth.split_outputs(out)

    for rnd in range(40):
        puts = [[synth.OP_PUT, int(rng.choice(ut)), int(rng.integers(0, 50)), 0, -1, 8, -1, 0, -1, -1]
                for _ in range(3000)]
        step(puts)
        for b in range(3):  # nearly every unit is taken and got: the round's pages die
            R = 1000
            ranks = rng.integers(0, A, size=R)
            types = np.full((R, 16), -2, np.int32)
            types[:, 0] = rng.choice(ut + [-1, -1, -1], size=R)
            outs = step(synth.reserve_events(ranks, types, np.zeros(R, np.int32)))
            gets = [[synth.OP_GET, int(r), int(x[5])] for r, x in zip(ranks, outs) if x[0] == 1]
            if gets:
                step(gets)
    st = {}
    with Server(ut, A, 1, 0, max_units=1 << 17) as s:
        s.set_param("recycle_pages", recycle)
        got = replay.replay(s, np.concatenate(trace))
        st = {k: s.stat(k) for k in ("pages_recycled", "open_pages", "pages_total")}
    assert_same(got, np.concatenate(exp))
    if recycle:
        assert st["pages_recycled"] > 0 and st["pages_total"] <= 12, st
    else:
        assert st["pages_recycled"] == 0, st


def _sparse_types(w, seed):
    """The workload with its declared type values spread over [0, 10010) (the reference's DBG arrays
    index by value below 10010, adlb.c:343-356), shuffled, and one value declared twice at the end
    (get_type_idx keeps the first index, adlb.c:3476-3485)."""
    rng = np.random.default_rng(seed)
    T = len(w.user_types)
    vals = rng.choice(10010, size=T, replace=False).astype(np.int32)
    remap = {int(a): int(b) for a, b in zip(w.user_types, vals)}
    w.u_type = vals[np.searchsorted(w.user_types, w.u_type)]
    rt = w.r_types.copy()
    m = rt >= 0
    rt[m] = vals[np.searchsorted(w.user_types, rt[m])]
    w.r_types = rt
    w.user_types = np.concatenate([vals, vals[:1]])
    assert len(remap) == T
    return w


CASES = {
    "c2_n200k_r16k": lambda: synth.config2(n_units=200_000, n_reserves=16_384, seed=201),
    "c2_eq_n200k_r16k": lambda: synth.config2(n_units=200_000, n_reserves=16_384, seed=202, equal_prio=True),
    "c2_t1": lambda: synth.config2(n_units=50_000, n_types=1, n_reserves=8192, seed=203),
    "c2_t64_wide": lambda: synth.config2(n_units=100_000, n_types=64, n_reserves=8192, seed=204,
                                         prio_hi=1 << 20),
    # some open pages wide (prio column read), the rest narrow (packed offsets)
    "c2_mixed_wide_pages": lambda: synth.config2(n_units=200_000, n_reserves=16_384, seed=209, wide_frac=1e-4),
    "c2_all_wide_pages": lambda: synth.config2(n_units=100_000, n_reserves=8192, seed=210, wide_frac=0.5),
    # the whole int32 range: INT_MAX next to ADLB_LOWEST_PRIO and below it (never matched)
    "c2_extreme_prios": lambda: synth.config2(n_units=60_000, n_reserves=8192, seed=212, wide_frac=0.05,
                                              wide_range=(-(1 << 31), (1 << 31) - 1)),
    "c2_exhaust": lambda: synth.config2(n_units=5_000, n_reserves=8192, seed=205, prio_hi=16),
    "c2_exhaust_nohang": lambda: synth.config2(n_units=5_000, n_reserves=8192, seed=206, hang=0),
    "c4_n200k": lambda: synth.config4(n_units=200_000, n_reserves=8192, n_ranks=256, seed=207),
    "c4_t8_tied": lambda: synth.config4(n_units=100_000, n_types=8, n_reserves=8192, n_ranks=64, seed=208,
                                        prio_hi=4),
    # T <= 8 with thresholds in multi-priority bins: k_select_open cannot rank, k_rank sorts and ranks
    "c2_t4_wide_prio": lambda: synth.config2(n_units=100_000, n_reserves=16_384, seed=230, prio_hi=1 << 20),
    "c2_t8_wide_prio": lambda: synth.config2(n_units=100_000, n_types=8, n_reserves=8192, seed=231,
                                             prio_hi=1 << 16),
    # more than 64 types: the sorted-runs Reserve path (adlbq_wide.hip), untargeted and targeted
    "w100_c2": lambda: synth.config2(n_units=50_000, n_types=100, n_reserves=8192, seed=240, prio_hi=128),
    "w150_c4": lambda: synth.config4(n_units=50_000, n_types=150, n_reserves=4096, n_ranks=128, seed=241,
                                     prio_hi=512),
    "w255_exhaust": lambda: synth.config2(n_units=4_000, n_types=255, n_reserves=6000, seed=242, prio_hi=8),
    # more than 255 types (get_type_idx has no bound, adlb.c:3476-3485): the type index's high bits in
    # meta, every page wide; declared values spread out, shuffled and repeated (first declared index wins)
    "w300_c2": lambda: synth.config2(n_units=60_000, n_types=300, n_reserves=8192, seed=243, prio_hi=256),
    "w300_c4": lambda: synth.config4(n_units=60_000, n_types=300, n_reserves=4096, n_ranks=128, seed=244,
                                     prio_hi=512),
    "w1000_sparse": lambda: _sparse_types(synth.config2(n_units=40_000, n_types=1000, n_reserves=6000, seed=245,
                                                        prio_hi=64), seed=246),
    # 8 < T <= 64 (keyrank): keys varying only in the bucket position, and over the whole int32 range
    "c2_t16_eq": lambda: synth.config2(n_units=100_000, n_types=16, n_reserves=8192, seed=233, equal_prio=True),
    "c2_t32_extreme": lambda: synth.config2(n_units=100_000, n_types=32, n_reserves=8192, seed=234, wide_frac=0.05,
                                            wide_range=(-(1 << 31), (1 << 31) - 1)),
    # a type with no unit at all (config 3's shards): the guess counts are adjusted first
    "c3_shard_missing_type": lambda: synth.config3_shard(1, 64, 80_000, 4, 8192, seed=232),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_fresh_vs_oracle(gpu_available, name):
    w = CASES[name]()
    tr = synth.workload_trace(w)
    cfg = (w.num_app_ranks, 1, 0)
    assert_same(run_abi(w.user_types, cfg, tr, max_units=w.n_units), run_oracle(w.user_types, cfg, tr))


VARIANTS = {
    "default": {},
    "rank_in_k_rank": {"rank_in_select": 0},  # k_rank ranks every candidate (k_select_open does not)
    "split_prep": {"split_prep": 1},          # request preparation and pass 1 as two launches
    "select_four_waves": {"select_wave": 0},  # pass 2 with four waves per page (k_select_open) for T <= 8
    "rank_launch": {"fuse_rank_chain": 0},    # k_rank as a launch of its own, not in the chain's (T <= 8)
    # k_rank's blocks in the chain's launch doing the ranking (k_select_open does not rank): the segments wait
    "fused_rank_ranks": {"rank_in_select": 0, "fuse_rank_chain": 1},
    # the pre-targeted match over the rank buckets' pages (k_targeted) / always the sorted index
    "targeted_scan": {"targeted_scan": 1},
    "targeted_index": {"targeted_scan": 0},
}


@pytest.mark.parametrize("name", ["c2_n200k_r16k", "c2_eq_n200k_r16k", "c2_mixed_wide_pages", "c2_exhaust",
                                  "c4_t8_tied", "c2_t1", "c2_t4_wide_prio", "c3_shard_missing_type"])
@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_pipeline_variants_vs_oracle(gpu_available, name, variant):
    """The scan and chain variants (adlbq_set_param) give the sequential result."""
    w = CASES[name]()
    tr = synth.workload_trace(w)
    cfg = (w.num_app_ranks, 1, 0)
    assert_same(run_abi(w.user_types, cfg, tr, max_units=w.n_units, params=VARIANTS[variant]),
                run_oracle(w.user_types, cfg, tr))


@pytest.mark.parametrize("name", ["c4_n200k", "c2_t64_wide", "c4_t8_tied"])
@pytest.mark.parametrize("grid", [1, 4])
def test_rank_small_grid_sorts_every_list(gpu_available, name, grid):
    """k_rank's in-launch list sort on a grid smaller than the number of lists to
    sort (the small grid a rank hint picks): each workgroup takes every grid-th
    list, so no sort wait is left hanging and the lists come out ordered."""
    w = CASES[name]()
    tr = synth.workload_trace(w)
    cfg = (w.num_app_ranks, 1, 0)
    got = run_abi(w.user_types, cfg, tr, max_units=w.n_units,
                  params={"rank_grid": grid, "keyrank": 0})
    assert_same(got, run_oracle(w.user_types, cfg, tr))


KEYRANK_MODES = {
    "on": {},
    "off": {"keyrank": 0},            # per-list sort + k_rank's searches
    "failover": {"keyrank_bin_max": 0},  # every binning fails over: k_rank sorts and ranks in its launch
}


@pytest.mark.parametrize("name", ["c4_n200k", "c2_t64_wide", "c2_t16_eq", "c2_t32_extreme"])
@pytest.mark.parametrize("mode", sorted(KEYRANK_MODES))
def test_keyrank_vs_oracle(gpu_available, name, mode):
    """8 < T <= 64: the lists sorted and ranked by one binning of the keys
    (adlbq_keyrank.hip), the sort + k_rank path, and a binning that fails over
    to k_rank inside the batch all give the sequential result."""
    w = CASES[name]()
    tr = synth.workload_trace(w)
    cfg = (w.num_app_ranks, 1, 0)
    st = {}
    got = run_abi(w.user_types, cfg, tr, max_units=w.n_units, params=KEYRANK_MODES[mode], stats=st)
    assert_same(got, run_oracle(w.user_types, cfg, tr))
    if mode == "on":
        # c2_t32_extreme: a few prios at the ends of the int32 range put the bulk of the keys
        # into one digit bin, so its first batch fails over (by design) and later ones skip keyrank
        assert st["keyrank"] >= 1 and (st["keyrank_failed"] == 0 or name == "c2_t32_extreme"), st
    elif mode == "off":
        assert st["keyrank"] == 0, st
    else:
        assert st["keyrank_failed"] >= 1, st


@pytest.mark.parametrize("variant", sorted(VARIANTS))
def test_pipeline_variants_depletion(gpu_available, variant):
    """Several Reserve batches in a row through each variant (the guessed cut,
    chunk sums and start guesses carry from batch to batch)."""
    w = synth.config2(n_units=30_000, n_reserves=4096, seed=311)
    rng = np.random.default_rng(9)
    parts = [synth.put_events(w)]
    for _ in range(5):
        parts.append(synth.reserve_events(w.r_rank, synth.type_vectors(rng, w.user_types, w.n_reserves), w.r_hang))
        parts.append(synth.simple_events(synth.OP_INFO))
    tr = np.concatenate(parts)
    cfg = (w.num_app_ranks, 1, 0)
    assert_same(run_abi(w.user_types, cfg, tr, max_units=w.n_units, params=VARIANTS[variant]),
                run_oracle(w.user_types, cfg, tr))


@pytest.mark.parametrize("name", ["c2_n200k_r16k", "c2_t64_wide", "c4_n200k", "c4_t8_tied"])
@pytest.mark.parametrize("passes", [1, 2, 3])
def test_chain_fixup_path(gpu_available, name, passes):
    """Few round launches (no warm-up) leave segments off their fixed point, so
    the last round's in-order walk re-solves them: still identical to the oracle."""
    w = CASES[name]()
    tr = synth.workload_trace(w)
    cfg = (w.num_app_ranks, 1, 0)
    st = {}
    got = run_abi(w.user_types, cfg, tr, max_units=w.n_units, params={"chain_passes": passes, "chain_warm": 0},
                  stats=st)
    assert_same(got, run_oracle(w.user_types, cfg, tr))
    if name == "c2_n200k_r16k" and passes == 1:
        assert st["chain_fallback"] > 0, st


@pytest.mark.parametrize("equal_prio", [False, True])
def test_depletion_batches_vs_oracle(gpu_available, equal_prio):
    """Reserve batches with nothing given back: each batch pins the best units,
    so the next one's thresholds sit deeper below the anchor (exact bins, then
    far bins and the sort path) while the anchor follows the live maximum."""
    w = synth.config2(n_units=20_000, n_reserves=4096, seed=211, equal_prio=equal_prio)
    rng = np.random.default_rng(5)
    parts = [synth.put_events(w)]
    for _ in range(4):
        tv = synth.type_vectors(rng, w.user_types, w.n_reserves)
        parts.append(synth.reserve_events(w.r_rank, tv, w.r_hang))
        parts.append(synth.simple_events(synth.OP_INFO))  # ends the batch
    tr = np.concatenate(parts)
    cfg = (w.num_app_ranks, 1, 0)
    assert_same(run_abi(w.user_types, cfg, tr, max_units=w.n_units), run_oracle(w.user_types, cfg, tr))


def test_stream_vs_oracle(gpu_available):
    o = oracle.Oracle("own")
    o.init([1, 2], 128, 8, 3)
    tr = synth.config5_stream(lambda ev: synth.split_outputs(o.replay(ev)), n_rounds=400, n_ranks=128,
                              n_servers=8, my_idx=3, seed=501)
    cfg = (128, 8, 3)
    assert_same(run_abi([1, 2], cfg, tr), run_oracle([1, 2], cfg, tr))


def test_stream_native_concurrent_vs_oracle(gpu_available):
    """Four shards' config-5 streams replayed at once by the native driver
    (adlb_replay.cpp: one host thread and HIP stream per shard, the bench's
    config-5 path): every shard's output equals the oracle's, and equals the
    Python driver's on the same handle type."""
    S, A = 4, 128
    traces, exp = [], []
    for j in range(S):
        o = oracle.Oracle("own", private=True)
        o.init([1, 2], A, S, j)
        tr = synth.config5_stream(lambda ev: synth.split_outputs(o.replay(ev)), n_rounds=120, n_ranks=A,
                                  n_servers=S, my_idx=j, seed=700 + j)
        traces.append(np.asarray(tr, np.int32))
        exp.append(run_oracle([1, 2], (A, S, j), tr))
    srvs = [Server([1, 2], A, S, j, max_units=1 << 16) for j in range(S)]
    try:
        got, calls = replay.replay_many(srvs, traces)
    finally:
        for s in srvs:
            s.close()
    for j in range(S):
        assert calls[j] > 0
        assert_same(got[j], exp[j])


def _exact_full(w, batches=1, stats=None, params=()):
    with Server(w.user_types, w.num_app_ranks, max_units=w.n_units) as s:
        for k, v in params:
            s.set_param(k, v)
        units = np.stack([w.u_type, w.u_prio, w.u_answer, w.u_target, w.u_len,
                          np.full(w.n_units, -1), np.zeros(w.n_units), np.full(w.n_units, -1),
                          np.full(w.n_units, -1)], axis=1).astype(np.int32)
        s.put_batch(units)
        reqs = np.concatenate([w.r_rank[:, None], w.r_hang[:, None].astype(np.int32), w.r_types],
                              axis=1).astype(np.int32)
        seq = np.arange(1, w.n_units + 1)
        avail = np.ones(w.n_units, bool)
        first = None
        for b in range(batches):
            resp = s.reserve_batch(reqs)
            check_batch(w.user_types, w.u_type, w.u_prio, w.u_target, seq, avail, w.r_rank, w.r_types,
                        w.r_hang, resp)
            if first is None:
                first = resp.copy()
            else:
                assert np.array_equal(first, resp), "same state + same batch must give the same answer"
            m = np.nonzero(resp[:, 0] == 1)[0]
            # return the units (SS_UNRESERVE) so the next batch sees the same queue
            if m.size:
                import torch
                trip = torch.tensor(np.stack([w.r_rank[m], resp[m, 5], np.full(m.size, -1)], axis=1)
                                    .astype(np.int32).ravel(), device="cuda")
                torch.cuda.synchronize()  # the handle's stream does not order after torch's
                s.unreserve_batch_device(m.size, trip.data_ptr())
                s.sync()
        if stats is not None:
            for k in ("device_sorted_lists", "sort_timeouts", "sort_radix", "sort_async_bad", "keyrank",
                      "keyrank_failed"):
                stats[k] = s.stat(k)
        return first


def test_full_size_config2_exact(gpu_available):
    w = synth.config2(n_units=10_000_000, n_reserves=65_536, seed=7)
    resp = _exact_full(w, batches=2)
    assert (resp[:, 0] == 1).all()


def test_full_size_config2_equal_prio_exact(gpu_available):
    w = synth.config2(n_units=10_000_000, n_reserves=65_536, seed=8, equal_prio=True)
    _exact_full(w)


@pytest.mark.parametrize("rounds", [-1, 1])
def test_config4_2m_exact(gpu_available, rounds):
    """Four batches through the per-list sort + k_rank path (keyrank off): the
    first batch's multi-prio-bin candidate lists are sorted after a read-back
    of their bounds (a device-wide radix sort per long list, one workgroup per
    short one); from the third batch on, by the hand-written list-stable radix
    sort planned from the last landed batch, without a read-back.  rounds:
    prefix-round launches of the 32-type ordered choice after round 0 (-1 =
    auto; 1 leaves the in-order walk more to do)."""
    w = synth.config4(n_units=2_000_000, n_reserves=65_536, n_ranks=1024, seed=9)
    stats = {}
    _exact_full(w, batches=4, stats=stats, params=[("chain_rounds", rounds), ("keyrank", 0)])
    assert stats["device_sorted_lists"] > 0, "the read-back sort did not run"
    assert stats["sort_radix"] >= 2 and stats["sort_async_bad"] == 0, stats
    assert stats["sort_timeouts"] == 0


@pytest.mark.parametrize("rounds", [-1, 0])
def test_config4_2m_keyrank_exact(gpu_available, rounds):
    """Four config-4 batches (32 types, thresholds in multi-prio bins) through
    keyrank: every batch binned and ranked without a failover."""
    w = synth.config4(n_units=2_000_000, n_reserves=65_536, n_ranks=1024, seed=9)
    stats = {}
    _exact_full(w, batches=4, stats=stats, params=[("chain_rounds", rounds)])
    assert stats["keyrank"] == 4 and stats["keyrank_failed"] == 0 and stats["sort_timeouts"] == 0, stats


def test_full_size_config4_exact(gpu_available):
    """Config 4 at its BASELINE size (10M units, 80% targeted over 1024 ranks,
    32 Zipf types, 65,536 Reserves of 1-4 types): three batches through keyrank."""
    w = synth.config4(n_units=10_000_000, n_reserves=65_536, n_ranks=1024, seed=10)
    stats = {}
    _exact_full(w, batches=3, stats=stats)
    assert stats["sort_timeouts"] == 0 and stats["keyrank"] >= 3 and stats["keyrank_failed"] == 0, stats


def test_full_size_config4_sort_path_exact(gpu_available):
    """The same through the per-list sort + k_rank path (keyrank off)."""
    w = synth.config4(n_units=10_000_000, n_reserves=65_536, n_ranks=1024, seed=10)
    stats = {}
    _exact_full(w, batches=3, stats=stats, params=[("keyrank", 0)])
    assert stats["sort_timeouts"] == 0 and stats["sort_radix"] >= 1, stats


REPEAT = {
    "c2": lambda: synth.config2(n_units=50_000, n_reserves=4096, seed=221),
    "c2_eq": lambda: synth.config2(n_units=50_000, n_reserves=4096, seed=222, equal_prio=True),
    # far prios below the bulk: wide pages, while the cuts stay in the exact bins
    "c2_mixed_wide_pages": lambda: synth.config2(n_units=50_000, n_reserves=4096, seed=223, wide_frac=3e-4,
                                                 wide_range=(-(1 << 30), -(1 << 29))),
    "c2_all_wide_pages": lambda: synth.config2(n_units=50_000, n_reserves=4096, seed=224, wide_frac=0.5),
    "c2_t64": lambda: synth.config2(n_units=50_000, n_types=64, n_reserves=4096, seed=225, prio_hi=1 << 20),
    "c4": lambda: synth.config4(n_units=50_000, n_reserves=4096, n_ranks=128, seed=226),
}


@pytest.mark.parametrize("name", sorted(REPEAT))
def test_repeated_batches_vs_oracle(gpu_available, name):
    """Four Reserve batches against one queue, each batch's matches given back
    (SS_UNRESERVE) before the next, as in the bench: from the second batch on
    the pass-1 guess (last cut less a margin) holds, so k_select_open reads the
    speculative lists; wide pages read the prio column, narrow ones the packed
    offsets.  Identical to the oracle, event for event."""
    w = REPEAT[name]()
    cfg = (w.num_app_ranks, 1, 0)
    o = oracle.Oracle("own")
    o.init(w.user_types, *cfg)
    trace, exp = [], []

    def step(ev):
        ev = np.asarray(ev, dtype=np.int32).ravel()
        out = o.replay(ev)
        trace.append(ev)
        exp.append(out)
        return synth.split_outputs(out)

    step(synth.put_events(w))
    R, nb = len(w.r_rank), 4
    for b in range(nb):
        lo, hi = b * R // nb, (b + 1) * R // nb
        outs = step(synth.reserve_events(w.r_rank[lo:hi], w.r_types[lo:hi], w.r_hang[lo:hi]))
        back = [[synth.OP_UNRESERVE, int(r), int(x[5]), -1] for r, x in zip(w.r_rank[lo:hi], outs) if x[0] == 1]
        assert back, "the batch matched nothing"
        step(back)
    st = {}
    got = run_abi(w.user_types, cfg, np.concatenate(trace), max_units=w.n_units, stats=st)
    assert_same(got, np.concatenate(exp))
    if name in ("c2", "c2_mixed_wide_pages"):
        # exact-bin cuts: the last batch's guess held (no threshold in a lump); on
        # this small dense queue page 0's near list may overflow (-entries), which
        # only sends pass 2 back to the page
        assert st["spec_lists"] == 1 or -100000 < st["spec_lists"] < 0, ("spec_lists", st["spec_lists"])


@pytest.mark.parametrize("trust", [1, 0])
def test_unreserve_resp_restores_queue(gpu_available, trust):
    """adlbq_unreserve_resp_device (SS_UNRESERVE of every unit a batch matched,
    read from the batch's own responses) leaves the queue as it was: the same
    batch then gets the same answers, which equal the oracle's.  trust=1: the
    unreserve straight after the batch takes the exact path from the batch's
    (slot, wqseqno) records ("unres_trust"); 0: the checked path."""
    import torch
    w = synth.config2(n_units=100_000, n_reserves=8192, seed=231)
    reqs = np.concatenate([w.r_rank[:, None], w.r_hang[:, None].astype(np.int32), w.r_types],
                          axis=1).astype(np.int32)
    exp = run_oracle(w.user_types, (w.num_app_ranks, 1, 0), np.concatenate(
        [synth.put_events(w), synth.reserve_events(w.r_rank, w.r_types, w.r_hang)]))
    exp = synth.split_outputs(exp)[-len(reqs):]
    with Server(w.user_types, w.num_app_ranks, max_units=w.n_units) as s:
        units = np.stack([w.u_type, w.u_prio, w.u_answer, w.u_target, w.u_len, np.full(w.n_units, -1),
                          np.zeros(w.n_units), np.full(w.n_units, -1), np.full(w.n_units, -1)],
                         axis=1).astype(np.int32)
        s.put_batch(units)
        s.set_param("unres_trust", trust)
        d_req = torch.from_numpy(reqs).cuda()
        d_resp = torch.empty((len(reqs), 12), dtype=torch.int32, device="cuda")
        outs = []
        torch.cuda.synchronize()
        for _ in range(3):
            s.reserve_batch_device(len(reqs), d_req.data_ptr(), d_resp.data_ptr())
            s.sync()
            outs.append(d_resp.cpu().numpy().copy())
            s.unreserve_resp_device(len(reqs), d_req.data_ptr(), d_resp.data_ptr())
            s.sync()
        assert s.stat("unres_trusted") == (3 if trust else 0)
        # a second unreserve of the same responses finds nothing pinned (the checked path: the first changed
        # the queue), and the queue still answers the same
        s.unreserve_resp_device(len(reqs), d_req.data_ptr(), d_resp.data_ptr())
        s.reserve_batch_device(len(reqs), d_req.data_ptr(), d_resp.data_ptr())
        s.sync()
        outs.append(d_resp.cpu().numpy().copy())
        assert s.stat("unres_trusted") == (3 if trust else 0)
        assert (outs[0][:, 0] == 1).all()
        for o in outs[1:]:
            assert np.array_equal(o, outs[0])
        assert np.array_equal(outs[0][:, :10], np.asarray(exp)[:, :10])


@pytest.mark.parametrize("between", ["none", "put", "get"])
def test_unreserve_resp_partial_vs_oracle(gpu_available, between):
    """Unreserve of a batch where some Reserves match and others do not (more
    Reserves than units), with nothing, a Put above every unit or a Get in
    between (those two take the checked path), then batches that deplete the
    queue: every answer equals the oracle's, stepped through the same events."""
    import torch
    w = synth.config2(n_units=3000, n_reserves=4096, seed=233)
    cfg = (w.num_app_ranks, 1, 0)
    hang = np.zeros(len(w.r_rank), np.int32)
    reqs = np.concatenate([w.r_rank[:, None], hang[:, None], w.r_types], axis=1).astype(np.int32)
    units = np.stack([w.u_type, w.u_prio, w.u_answer, w.u_target, w.u_len, np.full(w.n_units, -1),
                      np.zeros(w.n_units), np.full(w.n_units, -1), np.full(w.n_units, -1)],
                     axis=1).astype(np.int32)
    o = oracle.Oracle("own")
    o.init(w.user_types, *cfg)

    def step(ev):
        return synth.split_outputs(o.replay(np.asarray(ev, dtype=np.int32).ravel()))

    step(synth.put_events(w))
    with Server(w.user_types, w.num_app_ranks, max_units=w.n_units + 16) as s:
        s.set_param("small_pages", 0)  # the batch pipeline (a 3000-unit bucket would take k_reserve_small)
        s.put_batch(units)
        d_req = torch.from_numpy(reqs).cuda()
        d_resp = torch.empty((len(reqs), 12), dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        s.reserve_batch_device(len(reqs), d_req.data_ptr(), d_resp.data_ptr())
        s.sync()
        first = d_resp.cpu().numpy().copy()
        exp = np.asarray(step(synth.reserve_events(w.r_rank, w.r_types, hang)))
        assert np.array_equal(first[:, :10], exp[:, :10])
        m = first[:, 0] == 1
        assert 0 < m.sum() < len(reqs)
        back = [(int(r), int(x[5])) for r, x in zip(w.r_rank, first) if x[0] == 1]
        if between == "put":
            extra = units[:1].copy()
            extra[0, 1] = 10 ** 6  # above every unit: the anchor must follow it
            s.put_batch(extra)
            step(np.concatenate([[synth.OP_PUT], extra[0, :5], [-1, 0, -1, -1]]))
        elif between == "get":
            r, q = back.pop(0)  # fetched, so the oracle does not unreserve it
            s.get_reserved(r, q)
            step([synth.OP_GET, r, q])
        s.unreserve_resp_device(len(reqs), d_req.data_ptr(), d_resp.data_ptr())
        step([[synth.OP_UNRESERVE, r, q, -1] for r, q in back])
        assert s.stat("unres_trusted") == (1 if between == "none" else 0)
        for b in range(3):
            s.reserve_batch_device(len(reqs), d_req.data_ptr(), d_resp.data_ptr())
            s.sync()
            got = d_resp.cpu().numpy()
            exp = np.asarray(step(synth.reserve_events(w.r_rank, w.r_types, hang)))
            assert np.array_equal(got[:, :10], exp[:, :10]), f"batch {b} after the unreserve"


@pytest.mark.parametrize("seed", [62, 63])
def test_bytes_hwm_vs_oracle(gpu_available, seed):
    """The handle's byte accounting (adlbq_bytes, adlbq_put_check) over a random
    put / Reserve / get / rq-delete stream, high-water mark included: identical
    to the restatement (whose current count the reference pins: t14, t15)."""
    import gen_golden
    tr = gen_golden.bytes_stream(seed=seed, n_events=500, kind="own", hwm=True)
    cfg = (16, 3, 1)
    assert_same(run_abi([0, 1, 2], cfg, tr), run_oracle([0, 1, 2], cfg, tr))


@pytest.mark.parametrize("n_parked", [3000, 6000])
def test_put_side_fifo_vs_oracle(gpu_available, n_parked):
    """Put-side matching (FA_PUT_HDR, adlb.c:963-1046; rq_find_rank_queued_for_type,
    xq.c:388-405) on a large rq: Reserves of 1-2 types or the wildcard park on an
    empty queue, then batches of untargeted and targeted Puts take them first-fit
    in FIFO order.  3000 parked: the LDS-staged block kernel; 6000: beyond its
    4096 staging entries, the one-wave scan."""
    rng = np.random.default_rng(n_parked)
    ut = np.array([3, 5, 7, 9], np.int32)
    A = 8192
    ranks = rng.permutation(A)[:n_parked]
    tv = synth.type_vectors(rng, ut, n_parked)
    parts = [synth.reserve_events(ranks, tv, np.ones(n_parked, np.uint8)), synth.simple_events(synth.OP_INFO)]
    n_put = n_parked + 500
    w = synth.config2(n_units=n_put, n_reserves=1, seed=n_parked)
    w.u_type[:] = ut[rng.integers(0, 4, n_put)]
    tgt = rng.random(n_put) < 0.3
    w.u_target[:] = np.where(tgt, ranks[rng.integers(0, n_parked, n_put)], -1)
    w.u_target[rng.random(n_put) < 0.05] = A - 1  # targeted at a rank with nothing parked
    for lo in range(0, n_put, 700):  # several Put batches, each one adlbq_put_batch
        parts += [synth.put_events(w, lo, min(n_put, lo + 700)), synth.simple_events(synth.OP_INFO),
                  synth.simple_events(synth.OP_BYTES)]
    trace = np.concatenate(parts)
    cfg = (A, 1, 0)
    assert_same(run_abi(ut, cfg, trace, max_units=1 << 14), run_oracle(ut, cfg, trace))


@pytest.mark.parametrize("delta", [None, 0, 3000])
def test_targeted_index_incremental_vs_oracle(gpu_available, delta):
    """Targeted Puts between Reserve batches (config-4 shape at reduced size):
    the targeted index takes each batch's new units into a sorted delta index
    read beside the main one (delta=None: the default capacity; 3000: folded
    into the main index when full; 0: merged into the main index every time),
    no full rebuild after the first, and every batch equals the oracle's
    sequential wq_find_pre_targeted_hi_prio / wq_find_hi_prio."""
    w = synth.config4(n_units=40_000, n_reserves=4096, seed=91)
    cfg = (w.num_app_ranks, 1, 0)
    rng = np.random.default_rng(91)
    n0 = 30_000
    parts = [synth.put_events(w, 0, n0)]
    R, nb = w.n_reserves, 4
    lo_u = n0
    for b in range(nb):
        lo, hi = b * R // nb, (b + 1) * R // nb
        parts.append(synth.reserve_events(w.r_rank[lo:hi], w.r_types[lo:hi], np.zeros(hi - lo, np.uint8)))
        hi_u = min(w.n_units, lo_u + 2500)   # the next slice of units: ~80% targeted
        parts.append(synth.put_events(w, lo_u, hi_u))
        lo_u = hi_u
        parts.append(synth.simple_events(synth.OP_INFO))
    trace = np.concatenate(parts)
    with Server(w.user_types, *cfg, max_units=w.n_units) as s:
        if delta is not None:
            s.set_param("tindex_delta", delta)
        got = replay.replay(s, trace)
        merges, rebuilds = s.stat("tindex_merges"), s.stat("tindex_rebuilds")
        dmerges, folds = s.stat("tindex_delta_merges"), s.stat("tindex_folds")
    assert_same(got, run_oracle(w.user_types, cfg, trace))
    assert rebuilds <= 2 and merges + dmerges >= 2, (merges, dmerges, rebuilds)
    if delta == 0:
        assert dmerges == 0
    if delta == 3000:
        assert folds >= 1 and dmerges >= 1, (folds, dmerges)


@pytest.mark.parametrize("delta", [None, 0])
def test_targeted_index_delta_overflow_vs_oracle(gpu_available, delta):
    """One rank sends more Reserves in a batch than a targeted workgroup takes
    at once (TGT_REQ = 1024): its later Reserves resume after the last unit
    each type gave, across the main and the delta index alike."""
    rng = np.random.default_rng(17)
    ut = np.array([4, 9, 13], np.int32)
    A = 8
    n0, n1 = 6000, 1500
    def units(n, seed):
        r = np.random.default_rng(seed)
        tgt = np.where(r.random(n) < 0.9, r.integers(0, A, n), -1)
        return np.stack([ut[r.integers(0, 3, n)], r.integers(0, 200, n), r.integers(0, A, n), tgt,
                         np.ones(n), np.full(n, -1), np.zeros(n), np.full(n, -1), np.full(n, -1)],
                        axis=1).astype(np.int32)
    u0, u1 = units(n0, 3), units(n1, 4)
    R = 3000
    reqs = np.full((R, 18), -2, np.int32)
    reqs[:, 0] = np.where(rng.random(R) < 0.8, 2, rng.integers(0, A, R))  # rank 2: ~2400 Reserves
    reqs[:, 1] = 0
    k = rng.integers(1, 3, R)
    for j in range(R):
        reqs[j, 2:2 + k[j]] = rng.choice(ut, k[j], replace=False)
    def put_units(u):  # OP_PUT events of unit rows (type, prio, answer, target, len, 4 common fields)
        ev = np.empty((u.shape[0], 10), np.int32)
        ev[:, 0] = synth.OP_PUT
        ev[:, 1:] = u
        return ev.ravel()
    trace = np.concatenate([put_units(u0), synth.reserve_events(reqs[:500, 0], reqs[:500, 2:], reqs[:500, 1]),
                            put_units(u1),
                            synth.reserve_events(reqs[500:, 0], reqs[500:, 2:], reqs[500:, 1])])
    cfg = (A, 1, 0)
    with Server(ut, *cfg, max_units=n0 + n1) as s:
        if delta is not None:
            s.set_param("tindex_delta", delta)
        got = replay.replay(s, trace)
    assert_same(got, run_oracle(ut, cfg, trace))


def test_put_batch_device_matches_host_variant(gpu_available):
    """adlbq_put_batch_device (results left in device memory, nothing waits)
    gives the results adlbq_put_batch does, including Puts that take parked
    Reserves, and leaves the same queue behind (a Reserve batch after it)."""
    import torch
    rng = np.random.default_rng(5)
    ut = np.array([3, 5, 7], np.int32)
    A = 4096
    ranks = rng.permutation(A)[:1500]
    tv = synth.type_vectors(rng, ut, 1500)
    outs = []
    for dev_path in (False, True):
        with Server(ut, A, max_units=1 << 14) as s:
            s.reserve_batch(np.concatenate([ranks[:, None], np.ones((1500, 1), np.int32), tv], axis=1))
            got = []
            for b in range(4):
                w = synth.config2(n_units=600, n_reserves=1, seed=50 + b)
                units = np.stack([ut[rng.integers(0, 3, 600)], w.u_prio, w.u_answer,
                                  np.where(rng.random(600) < 0.3, ranks[rng.integers(0, 1500, 600)], -1), w.u_len,
                                  np.full(600, -1), np.zeros(600), np.full(600, -1), np.full(600, -1)],
                                 axis=1).astype(np.int32)
                if dev_path:
                    d = torch.empty((600, 3), dtype=torch.int32, device="cuda")
                    s.put_batch_device(units, d.data_ptr())
                    s.sync()
                    got.append(d.cpu().numpy())
                else:
                    got.append(s.put_batch(units))
            tv2 = synth.type_vectors(rng, ut, 512)
            got.append(s.reserve_batch(np.concatenate([np.arange(512)[:, None], np.zeros((512, 1), np.int32), tv2],
                                                      axis=1)))
            got.append(np.asarray(s.info(), np.int64))
        outs.append(got)
        rng = np.random.default_rng(5)  # the same draws for the second pass
        ranks = rng.permutation(A)[:1500]
        tv = synth.type_vectors(rng, ut, 1500)
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)



ONE = {
    "one_c2_t4": lambda: synth.config2(n_units=30_000, n_reserves=300, seed=701),
    "one_c2_t8_wide": lambda: synth.config2(n_units=25_000, n_types=8, n_reserves=300, seed=702, wide_frac=0.2,
                                            wide_range=(-(1 << 31), (1 << 31) - 1)),
    "one_c2_t1_eq": lambda: synth.config2(n_units=20_000, n_types=1, n_reserves=300, seed=703, equal_prio=True),
    "one_c2_t3_tied": lambda: synth.config2(n_units=24_000, n_types=3, n_reserves=300, seed=704, prio_hi=3),
}


def _one_big(prio_hi, missing):
    """More page pairs than k_reserve_one's 256 workgroups (4.3M units, 1,050 pages).  prio_hi 2^20: a
    priority is rare, so once the best unit is taken the anchor is stale and no workgroup may stop
    early; missing: no unit of the last type (its Reserves never resolve early either)."""
    w = synth.config2(n_units=4_300_000, n_reserves=60, seed=707 + prio_hi % 97, prio_hi=prio_hi)
    if missing:
        w.u_type[w.u_type == w.user_types[-1]] = w.user_types[0]
    return w


ONE_BIG = {"one_big_dense": lambda: _one_big(1024, False), "one_big_sparse": lambda: _one_big(1 << 20, False),
           "one_big_missing": lambda: _one_big(1024, True)}


@pytest.mark.parametrize("name", sorted(ONE_BIG))
def test_single_reserve_large_bucket_vs_oracle(gpu_available, name):
    """k_reserve_one stepping its 256 workgroups through 1,050 pages in bucket order, stopping once every
    wanted type's best unit sits at its anchor's priority before the next pair: single Reserves, nothing
    returned in between (pins accumulate), equal to the oracle Reserve after Reserve."""
    w = ONE_BIG[name]()
    parts = [synth.put_events(w)]
    for j in range(w.r_rank.size):
        parts.append(synth.reserve_events(w.r_rank[j:j + 1], w.r_types[j:j + 1], w.r_hang[j:j + 1]))
        parts.append(synth.simple_events(synth.OP_INFO))
    tr = np.concatenate(parts)
    cfg = (w.num_app_ranks, 1, 0)
    with Server(w.user_types, *cfg, max_units=w.n_units) as s:
        got = replay.replay(s, tr)
        assert s.stat("one_batches") == w.r_rank.size
    assert_same(got, run_oracle(w.user_types, cfg, tr))


@pytest.mark.parametrize("engine", ["one", "pipeline"])
@pytest.mark.parametrize("name", sorted(ONE))
def test_single_reserve_batches_vs_oracle(gpu_available, name, engine):
    """Batches of one Reserve on an open bucket larger than the one-workgroup
    path takes: k_reserve_one (one launch) and the pipeline both give the
    oracle's result, Reserve after Reserve (an INFO ends every batch)."""
    w = ONE[name]()
    parts = [synth.put_events(w)]
    for j in range(w.r_rank.size):
        parts.append(synth.reserve_events(w.r_rank[j:j + 1], w.r_types[j:j + 1], w.r_hang[j:j + 1]))
        parts.append(synth.simple_events(synth.OP_INFO))
    tr = np.concatenate(parts)
    cfg = (w.num_app_ranks, 1, 0)
    with Server(w.user_types, *cfg, max_units=w.n_units) as s:
        if engine == "pipeline":
            s.set_param("reserve_one", 0)
        got = replay.replay(s, tr)
        used = s.stat("one_batches")
    assert_same(got, run_oracle(w.user_types, cfg, tr))
    assert (used == w.r_rank.size) == (engine == "one"), used


def test_single_reserve_exhaustion_parks_vs_oracle(gpu_available):
    """One-Reserve batches past the end of the queue: the last ones find nothing
    and park (hang) or answer NO_CURR_WORK, as the oracle does."""
    w = synth.config2(n_units=20_100, n_types=2, n_reserves=40, seed=705, prio_hi=5)
    parts = [synth.put_events(w)]
    # take nearly everything in one batch first, then single Reserves run the queue dry
    big = 20_080
    rng = np.random.default_rng(706)
    tv = synth.type_vectors(rng, w.user_types, big)
    parts.append(synth.reserve_events(np.arange(big) % w.num_app_ranks, tv, np.ones(big, np.uint8)))
    parts.append(synth.simple_events(synth.OP_INFO))
    for j in range(w.r_rank.size):
        parts.append(synth.reserve_events(w.r_rank[j:j + 1], w.r_types[j:j + 1], w.r_hang[j:j + 1]))
        parts.append(synth.simple_events(synth.OP_INFO))
    tr = np.concatenate(parts)
    cfg = (w.num_app_ranks, 1, 0)
    with Server(w.user_types, *cfg, max_units=w.n_units) as s:
        s.set_param("recycle_pages", 0)  # the emptied pages stay open: the bucket stays above four pages
        got = replay.replay(s, tr)
        used = s.stat("one_batches")
    assert_same(got, run_oracle(w.user_types, cfg, tr))
    assert used == w.r_rank.size, used


@pytest.mark.parametrize("T", [4, 8])
def test_one_and_pipeline_batches_interleaved_vs_oracle(gpu_available, T):
    """k_reserve_one (one-Reserve batches) alternating with pipeline batches of
    ~1024 Reserves and Put batches on an open bucket of more than 10 pages: the
    state one path leaves for the other (anchors, guessed cuts, the landed
    snapshot's plan / keyrank / rank hints) never changes a result."""
    rng = np.random.default_rng(80 + T)
    ut, A = np.arange(T, dtype=np.int32), 2048
    o = oracle.Oracle("own")
    o.init(ut, A, 1, 0)
    trace, exp = [], []

    def step(ev):
        ev = np.asarray(ev, dtype=np.int32).ravel()
        out = o.replay(ev)
        trace.append(ev)
        exp.append(out)
        return synth.split_outputs(out)

    def puts(n):
        return [[synth.OP_PUT, int(rng.choice(ut)), int(rng.integers(0, 200)), 0, -1, 8, -1, 0, -1, -1]
                for _ in range(n)]

    def reserves(R):
        ranks = rng.integers(0, A, size=R)
        return ranks, step(synth.reserve_events(ranks, synth.type_vectors(rng, ut, R), np.ones(R, np.uint8)))

    step(puts(50_000))  # 13 pages
    for rnd in range(30):
        for R in (1, 1024, 1, 1, 700, 1):
            ranks, outs = reserves(R)
            if rnd % 3 == 2:  # Gets of some matches: units leave the bucket
                gets = [[synth.OP_GET, int(r), int(x[5])] for r, x in zip(ranks, outs) if x[0] == 1][::2]
                if gets:
                    step(gets)
        step(puts(int(rng.integers(200, 1500))))
    with Server(ut, A, 1, 0, max_units=1 << 17) as s:
        got = replay.replay(s, np.concatenate(trace))
        assert s.stat("one_batches") > 0
    assert_same(got, np.concatenate(exp))


@pytest.mark.parametrize("mode", [1, 0, 8])
@pytest.mark.parametrize("name", ["s_c4_targeted", "s_c4_t8_tied", "s_c4_r256"])
def test_targeted_scan_vs_index_small(gpu_available, name, mode):
    """Small queues with targeted units: the pre-targeted match (xq.c:219-247) by
    scanning each rank bucket (k_targeted, "targeted_scan" 1) and by the sorted
    index (k_targeted_idx, 0: one Reserve at a time; 8: 64 Reserves of a bucket
    at a time by Jacobi rounds), each with the one-workgroup choice after it."""
    w = SMALL[name]()
    tr = synth.workload_trace(w)
    cfg = (w.num_app_ranks, 1, 0)
    with Server(w.user_types, *cfg, max_units=w.n_units) as s:
        s.set_param("targeted_scan", 1 if mode == 1 else 0)
        if mode == 8:
            s.set_param("targeted_diag", 8)
        got = replay.replay(s, tr)
        assert (s.stat("tscan_batches") > 0) == (mode == 1)
    assert_same(got, run_oracle(w.user_types, cfg, tr))


def test_config4_2m_targeted_blocks_exact(gpu_available):
    """The pre-targeted match served 64 Reserves of a bucket at a time by Jacobi
    rounds ("targeted_diag" 8) instead of one by one: the same exact answers."""
    w = synth.config4(n_units=2_000_000, n_reserves=65_536, n_ranks=1024, seed=9)
    stats = {}
    _exact_full(w, batches=3, stats=stats, params=[("targeted_diag", 8)])
    assert stats["sort_timeouts"] == 0, stats
