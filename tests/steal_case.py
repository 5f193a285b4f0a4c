"""Shared cases for the steal-round tests.

build_case() makes S config-3 shards (adlb_amd.synth.config3_shard at small
sizes, plus units targeted at ranks homed on the same shard and a few units at
ADLB_LOWEST_PRIO), replays Puts then Reserves on one private oracle per shard,
and returns the oracles with the per-shard event arrays.  ListShard is a
numpy model of a shard's exports (what adlbq_steal_export / adlbq_rq_export
compute on the device, restated by sorting) for the CPU-only merge tests.
"""
import numpy as np

import oracle
from adlb_amd import synth

LOWEST = synth.LOWEST_PRIO


def shard_workloads(S, n_units, R, seed, T=4, p_remote=0.3, prio_hi=64):
    ws = []
    for s in range(S):
        w = synth.config3_shard(s, S, n_units, T, R, seed, prio_hi, p_remote)
        rng = np.random.default_rng(seed * 31 + s)
        # targeted units: only at ranks homed on this shard (rank % S == s), whose
        # Reserves come here -- the pre-targeted match stays local (module doc)
        tg = rng.random(n_units) < 0.05
        w.u_target[tg] = (rng.integers(0, R, int(tg.sum())) * S + s).astype(np.int32)
        w.u_prio[rng.random(n_units) < 0.01] = LOWEST
        ws.append(w)
    return ws


def build_case(S, n_units, R, seed, **kw):
    ws = shard_workloads(S, n_units, R, seed, **kw)
    orcs, resps = [], []
    for s, w in enumerate(ws):
        o = oracle.Oracle("own", private=True)
        o.init(w.user_types, w.num_app_ranks, S, s)
        out = synth.split_outputs(o.replay(synth.workload_trace(w)))
        resps.append(np.asarray(out[w.n_units:], dtype=np.int32))
        orcs.append(o)
    return ws, orcs, resps


class ListShard:
    """TEST MODEL: one shard's available units and parked Reserves as arrays."""

    def __init__(self, w, idx, S, resp, rq):
        self.user_types = w.user_types
        self.T = int(w.user_types.size)
        self.num_app_ranks = w.num_app_ranks
        self.num_servers = S
        self.my_server_idx = idx
        n = w.n_units
        self.seq = np.arange(1, n + 1, dtype=np.int32)
        self.w = w
        self.avail = (w.u_target < 0) & (w.u_prio > LOWEST)
        self.avail[resp[resp[:, 0] == 1, 5] - 1] = False
        self.rq = np.asarray(rq, dtype=np.int32).reshape(-1, 18).copy()

    def steal_export(self, k):
        T, w = self.T, self.w
        recs = np.zeros((T, k, 8), np.int32)
        nrec = np.zeros(T, np.int32)
        navail = np.zeros(T, np.int64)
        for t in range(T):
            idx = np.nonzero(self.avail & (w.u_type == self.user_types[t]))[0]
            idx = idx[np.lexsort((self.seq[idx], -w.u_prio[idx].astype(np.int64)))]
            navail[t] = idx.size
            top = idx[:k]
            nrec[t] = top.size
            recs[t, :top.size] = np.stack([w.u_prio[top], self.seq[top], w.u_type[top], w.u_len[top],
                                           w.u_answer[top], np.zeros(top.size), np.full(top.size, -1),
                                           np.full(top.size, -1)], axis=1)
        return recs, nrec, navail

    def rq_export(self):
        return self.rq.copy()

    def steal_begin(self, k):
        self._k = k

    def steal_collect(self):
        return (*self.steal_export(self._k), self.rq_export())

    def steal_apply(self, pairs, rqseqnos):
        self._bad = (int((self.grant_batch(pairs) == 0).sum()), int((self.rq_delete_batch(rqseqnos) == 0).sum()))

    def steal_check(self):
        bad, self._bad = getattr(self, "_bad", (0, 0)), (0, 0)
        return bad

    def grant_batch(self, pairs):
        found = np.zeros(len(pairs), np.int32)
        for i, (rank, seq) in enumerate(np.asarray(pairs).reshape(-1, 2)):
            if 0 < seq <= self.seq.size and self.avail[seq - 1]:
                self.avail[seq - 1] = False
                found[i] = 1
        return found

    def rq_delete_batch(self, rqseqnos):
        rqs = np.asarray(rqseqnos).ravel()
        found = np.isin(rqs, self.rq[:, 0]).astype(np.int32)
        self.rq = self.rq[~np.isin(self.rq[:, 0], rqs)]
        return found


def list_shards(ws, orcs, resps):
    return [ListShard(w, s, len(ws), resps[s], orcs[s].rq_list()) for s, w in enumerate(ws)]


def rounds(round_fn, max_rounds=10_000):
    """Repeat a steal round until it settles nothing more (over all shards: a
    round that settles anything consumed an exported unit, so a round that
    stops early always makes progress); concatenated responses."""
    got = []
    for _ in range(max_rounds):
        r = round_fn()
        got.append(r.resp)
        if r.settled == 0:
            break
    return np.concatenate(got) if got else np.zeros((0, 15), np.int32)
