"""Seeded synthetic workloads for the ADLB server queue.

Everything here is plain numpy and deterministic in ``seed``.  The same arrays
feed (a) the event traces replayed by the oracle / the product replayer and
(b) the benchmark, so the benchmark's inputs are exactly the parity-tested
shapes.

Request type vectors are built the way the client stub normalises them before
they reach the server (``adlbp_Reserve``, adlb.c:2903-2916): the listed types,
then ``-2`` padding; a wildcard request is ``[-1, -2, -2, ...]``.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

REQ_TYPES = 16               # REQ_TYPE_VECT_SZ, xq.h:37
LOWEST_PRIO = -999999999     # ADLB_LOWEST_PRIO, adlb.h:22
OP_PUT, OP_RESERVE, OP_GET, OP_UNRESERVE = 1, 2, 3, 4
OP_QMROW, OP_SETROW, OP_CHECKREM, OP_RFRDONE, OP_TQADD = 5, 6, 7, 8, 9
OP_PUSHSEL, OP_INFO, OP_RQDEL, OP_INFOTYPE = 10, 11, 12, 13
OP_PUSHACCEPT, OP_PUSHTAKE, OP_PUSHCOMMIT, OP_PUSHDEL = 19, 20, 21, 22  # the SS_PUSH_* handlers (adlb.c:2109-2362)
OP_BYTES, OP_PUTCHECK, OP_HWM = 16, 17, 18  # queue bytes beyond init; FA_PUT_HDR memory check (work_len, max_malloc); their high-water mark


@dataclass
class Workload:
    """A server's configuration plus a unit population and a Reserve batch."""
    user_types: np.ndarray            # (T,) int32 user type values
    num_app_ranks: int
    # units, in Put (== wqseqno) order
    u_type: np.ndarray                # user type value
    u_prio: np.ndarray
    u_target: np.ndarray              # -1 untargeted
    u_answer: np.ndarray
    u_len: np.ndarray
    # reserves, in arrival order
    r_rank: np.ndarray
    r_types: np.ndarray               # (R, 16)
    r_hang: np.ndarray                # (R,) uint8
    name: str = ""
    meta: dict = field(default_factory=dict)

    @property
    def n_units(self) -> int:
        return int(self.u_type.size)

    @property
    def n_reserves(self) -> int:
        return int(self.r_rank.size)


# ----------------------------------------------------------------------------- trace encoding
def put_events(w: Workload, lo: int = 0, hi: int | None = None) -> np.ndarray:
    hi = w.n_units if hi is None else hi
    n = hi - lo
    ev = np.empty((n, 10), dtype=np.int32)
    ev[:, 0] = OP_PUT
    ev[:, 1] = w.u_type[lo:hi]
    ev[:, 2] = w.u_prio[lo:hi]
    ev[:, 3] = w.u_answer[lo:hi]
    ev[:, 4] = w.u_target[lo:hi]
    ev[:, 5] = w.u_len[lo:hi]
    ev[:, 6] = -1      # home_server_rank
    ev[:, 7] = 0       # common_len
    ev[:, 8] = -1      # common_server_rank
    ev[:, 9] = -1      # common_server_commseqno
    return ev.ravel()


def reserve_events(ranks, types16, hang) -> np.ndarray:
    ranks = np.asarray(ranks, dtype=np.int32)
    n = ranks.size
    ev = np.empty((n, 19), dtype=np.int32)
    ev[:, 0] = OP_RESERVE
    ev[:, 1] = ranks
    ev[:, 2] = np.asarray(hang, dtype=np.int32)
    ev[:, 3:] = np.asarray(types16, dtype=np.int32).reshape(n, REQ_TYPES)
    return ev.ravel()


def simple_events(op: int, *args) -> np.ndarray:
    return np.asarray([op, *args], dtype=np.int32)


def workload_trace(w: Workload) -> np.ndarray:
    return np.concatenate([put_events(w), reserve_events(w.r_rank, w.r_types, w.r_hang)])


# ----------------------------------------------------------------------------- request vectors
def type_vectors(rng, user_types, R, p_single=0.7, p_pair=0.2, p_wild=0.1,
                 weights=None, ntypes_range=None) -> np.ndarray:
    """(R, 16) request type vectors as normalised by the client stub."""
    T = len(user_types)
    out = np.full((R, REQ_TYPES), -2, dtype=np.int32)
    ut = np.asarray(user_types, dtype=np.int32)
    if ntypes_range is not None:
        lo, hi = ntypes_range
        k = rng.integers(lo, hi + 1, size=R)
        for j in range(R):
            kk = min(int(k[j]), T)
            out[j, :kk] = ut[rng.choice(T, kk, replace=False, p=weights)]
        return out
    u = rng.random(R)
    single = u < p_single
    pair = (u >= p_single) & (u < p_single + p_pair)
    wild = ~(single | pair)
    idx = rng.choice(T, size=R, p=weights)
    out[single, 0] = ut[idx[single]]
    npair = int(pair.sum())
    if npair:
        if T >= 2:
            a = rng.choice(T, size=npair, p=weights)
            off = rng.integers(1, T, size=npair)
            b = (a + off) % T
            out[pair, 0] = ut[a]
            out[pair, 1] = ut[b]
        else:
            out[pair, 0] = ut[0]
    out[wild, 0] = -1
    return out


def zipf_weights(T: int, s: float = 1.1) -> np.ndarray:
    w = 1.0 / np.arange(1, T + 1) ** s
    return w / w.sum()


# ----------------------------------------------------------------------------- configs
def config2(n_units=1_000_000, n_types=4, n_reserves=65_536, seed=2, prio_hi=1024,
            equal_prio=False, hang=1, wide_frac=0.0, wide_range=(-(1 << 30), 1 << 30)) -> Workload:
    """Config 2 / metric: untargeted units, uniform types, prio ~ U[0,prio_hi),
    R hanging Reserves from ranks 0..R-1 (70% one type, 20% two, 10% wildcard).
    wide_frac: that fraction of the units instead draws prio ~ U[wide_range)
    (pages whose prios span more than the packed-offset range)."""
    rng = np.random.default_rng(seed)
    ut = np.arange(n_types, dtype=np.int32)
    u_type = ut[rng.integers(0, n_types, size=n_units)]
    u_prio = (np.zeros(n_units, np.int32) if equal_prio
              else rng.integers(0, prio_hi, size=n_units).astype(np.int32))
    if wide_frac > 0:
        far = rng.random(n_units) < wide_frac
        u_prio[far] = rng.integers(wide_range[0], wide_range[1], size=int(far.sum())).astype(np.int32)
    R = n_reserves
    w = Workload(user_types=ut, num_app_ranks=max(R, 1),
                 u_type=u_type, u_prio=u_prio,
                 u_target=np.full(n_units, -1, np.int32),
                 u_answer=(np.arange(n_units) % max(R, 1)).astype(np.int32),
                 u_len=(8 + (np.arange(n_units) % 57)).astype(np.int32),
                 r_rank=np.arange(R, dtype=np.int32),
                 r_types=type_vectors(rng, ut, R),
                 r_hang=np.full(R, hang, np.uint8),
                 name="config2", meta=dict(seed=seed, prio_hi=prio_hi, equal_prio=equal_prio))
    return w


def config4(n_units=10_000_000, n_types=32, n_reserves=65_536, n_ranks=1024, seed=4,
            frac_targeted=0.8, prio_hi=1 << 16, hang=1) -> Workload:
    """Config 4: skewed targeted puts (80% targeted, target ~ Zipf(1.1) over A
    ranks), 32 types with Zipf(1.1) popularity, prio ~ U[0,2^16), Reserves from
    ranks U[0,A) with 1-4 types each, no wildcard."""
    rng = np.random.default_rng(seed)
    ut = np.arange(n_types, dtype=np.int32)
    tw = zipf_weights(n_types)
    u_type = ut[rng.choice(n_types, size=n_units, p=tw)]
    u_prio = rng.integers(0, prio_hi, size=n_units).astype(np.int32)
    targeted = rng.random(n_units) < frac_targeted
    rw = zipf_weights(n_ranks)
    u_target = np.where(targeted, rng.choice(n_ranks, size=n_units, p=rw), -1).astype(np.int32)
    R = n_reserves
    return Workload(user_types=ut, num_app_ranks=n_ranks, u_type=u_type, u_prio=u_prio,
                    u_target=u_target,
                    u_answer=(np.arange(n_units) % n_ranks).astype(np.int32),
                    u_len=(16 + (np.arange(n_units) % 101)).astype(np.int32),
                    r_rank=rng.integers(0, n_ranks, size=R).astype(np.int32),
                    r_types=type_vectors(rng, ut, R, weights=tw, ntypes_range=(1, 4)),
                    r_hang=np.full(R, hang, np.uint8),
                    name="config4", meta=dict(seed=seed))


def config3_types(rng, n_types, shard, R, p_remote=0.1) -> np.ndarray:
    """Config 3 Reserve type vectors of one shard: a fraction p_remote ask for
    just the shard's missing type (shard % T), the rest draw from its local
    types like config 2."""
    ut = np.arange(n_types, dtype=np.int32)
    miss = shard % n_types
    local = np.delete(ut, miss) if n_types > 1 else ut
    r_types = type_vectors(rng, local, R)
    remote = rng.random(R) < p_remote
    r_types[remote] = -2
    r_types[remote, 0] = miss
    return r_types


def config3_shard(shard, n_shards=64, n_units=1_562_500, n_types=4, n_reserves=8192, seed=3, prio_hi=1024,
                  p_remote=0.1, hang=1) -> Workload:
    """Config 3: one server shard of a queue sharded over n_shards servers
    (per-server seqnos).  Type popularity is skewed per shard: shard s holds no
    unit of type s % T, and a fraction p_remote of its Reserves ask for just
    that type -- no local match, so they park and go to the cross-shard steal
    round.  The other Reserves draw from the local types like config 2 (70% one
    type, 20% two, 10% wildcard).  Reserve j of shard s comes from app rank
    j * n_shards + s, so ranks are distinct across shards."""
    rng = np.random.default_rng(seed + 7919 * shard)
    ut = np.arange(n_types, dtype=np.int32)
    miss = shard % n_types
    local = np.delete(ut, miss) if n_types > 1 else ut
    u_type = local[rng.integers(0, local.size, size=n_units)]
    u_prio = rng.integers(0, prio_hi, size=n_units).astype(np.int32)
    R = n_reserves
    r_types = config3_types(rng, n_types, shard, R, p_remote)
    A = R * n_shards
    return Workload(user_types=ut, num_app_ranks=A, u_type=u_type, u_prio=u_prio,
                    u_target=np.full(n_units, -1, np.int32),
                    u_answer=(np.arange(n_units) % A).astype(np.int32),
                    u_len=(8 + (np.arange(n_units) % 57)).astype(np.int32),
                    r_rank=(np.arange(R) * n_shards + shard).astype(np.int32),
                    r_types=r_types, r_hang=np.full(R, hang, np.uint8),
                    name="config3", meta=dict(seed=seed, shard=shard, n_shards=n_shards, missing_type=int(miss)))


# ----------------------------------------------------------------------------- config 5: stream
def split_outputs(out: np.ndarray):
    """Split a replay output stream into per-event int arrays."""
    res, i, o = [], 0, out.tolist()
    while i < len(o):
        n = o[i]
        res.append(o[i + 1:i + 1 + n])
        i += 1 + n
    return res


def config5_stream(step, user_types=(1, 2), n_ranks=64, n_rounds=200, n_servers=4,
                   my_idx=0, seed=5, n_seed_units=512):
    """tsp.c-style branch-and-bound stream, driven by
    ``step(events) -> per-event outputs`` so the trace can react to outcomes
    (GETs name the wqseqno a Reserve returned).  Work units: type 1 untargeted,
    prio 1+len (tsp.c:240-241); bound updates: type 2 targeted, prio 999999999
    (tsp.c:17,189-193); Reserves ask for {2, 1} (tsp.c:157-161), some for
    {1} or the wildcard, 10% non-hanging.  Every few rounds: qmstat self-row,
    remote rows, steal round (check_remote), tq updates, RFR completions, push
    selection, unreserves and info queries.  Returns the full trace."""
    rng = np.random.default_rng(seed)
    ut = list(user_types)
    T = len(ut)
    W, B = ut[0], ut[-1]
    master = n_ranks
    trace = []

    def emit(ev):
        ev = np.asarray(ev, dtype=np.int32).ravel()
        trace.append(ev)
        return step(ev)

    def put_ev(t, prio, target, ln):
        return [OP_PUT, t, prio, int(rng.integers(0, n_ranks)), target, ln, -1, 0, -1, -1]

    emit(np.concatenate([put_ev(W, 1 + int(l), -1, int(l)) for l in rng.integers(4, 40, n_seed_units)]))
    holding = {}            # rank -> wqseqno reserved for it
    parked = set()
    for rnd in range(n_rounds):
        idle = [r for r in range(n_ranks) if r not in holding and r not in parked]
        rng.shuffle(idle)
        idle = idle[: max(1, len(idle) // 2)]
        if idle:
            ev = []
            for r in idle:
                u = rng.random()
                tv = [-2] * REQ_TYPES
                if u < 0.75:
                    tv[0], tv[1] = B, W
                elif u < 0.9:
                    tv[0] = W
                else:
                    tv[0] = -1
                ev += [OP_RESERVE, r, int(rng.random() < 0.9)] + tv
            outs = emit(ev)
            for r, o in zip(idle, outs):
                if o[0] == 1:
                    holding[r] = o[5]
                elif o[0] == 0:
                    parked.add(r)
        # workers fetch their units (a few unreserve instead)
        ev, who = [], []
        for r, seq in list(holding.items()):
            if rng.random() < 0.03:
                ev += [OP_UNRESERVE, r, seq, -1]
                who.append((r, 'u'))
            else:
                ev += [OP_GET, r, seq]
                who.append((r, 'g'))
        outs = emit(ev) if ev else []
        done = []
        for (r, kind), o in zip(who, outs):
            del holding[r]
            if kind == 'g' and o[0] == 1:
                done.append((r, o[2]))
        # each finished worker puts children and occasionally a bound update
        ev = []
        for r, t in done:
            if t == W:
                for l in rng.integers(4, 60, int(rng.integers(0, 4))):
                    ev += put_ev(W, 1 + int(l), -1, int(l))
            if rng.random() < 0.15:
                for tgt in rng.integers(0, n_ranks, int(rng.integers(1, 3))):
                    ev += put_ev(B, 999999999, int(tgt), 8)
        if not ev and not holding and rng.random() < 0.5:
            ev = put_ev(W, int(rng.integers(1, 50)), -1, 16)
        if ev:
            outs = emit(ev)
            for o in outs:
                if o[1] >= 0:          # matched a parked Reserve: that rank now holds it
                    parked.discard(o[1])
                    holding[o[1]] = o[0]
        # periodic server-side events
        if rnd % 5 == 4:
            emit([OP_QMROW])
            ev = []
            for i in range(n_servers):
                if i == my_idx:
                    continue
                hi = [int(x) if rng.random() < 0.7 else LOWEST_PRIO
                      for x in rng.integers(0, 1000, T)]
                ev += [OP_SETROW, i, int(rng.integers(0, 5)), int(rng.integers(0, 10 ** 6))] + hi
            if ev:
                emit(ev)
            outs = emit([OP_CHECKREM])
        if rnd % 7 == 3 and parked:
            r = int(rng.choice(sorted(parked)))
            srv = master + int(rng.integers(0, n_servers))
            emit([OP_TQADD, r, B, srv])
        if rnd % 3 == 1:
            srv = master + int(rng.integers(0, n_servers))
            emit([OP_RFRDONE, srv, int(rng.integers(0, n_ranks))])
        if rnd % 11 == 5:
            emit([OP_PUSHSEL, int(rng.integers(0, 10 ** 6))])
            emit([OP_INFO])
            emit([OP_INFOTYPE, W])
    return np.concatenate(trace)
