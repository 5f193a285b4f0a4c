"""The steal round on HIP shards against the oracle.

S server handles share the one GPU (one per shard, as a process holding
several servers would).  Each replays the same Puts and Reserves as its
oracle shard (responses compared), then steal rounds -- adlbq_steal_export
on the device, adlbq_steal_merge, adlbq_grant_batch / adlbq_rq_delete_batch --
must settle exactly what oracle.serial_steal_round settles, and leave every
shard in the oracle's state (qmstat row, counts, and a further Reserve batch).
"""
import numpy as np
import pytest

import oracle
from adlb_amd import replay, shards, synth
from adlb_amd.server import Server
from steal_case import build_case, rounds

pytestmark = pytest.mark.gpu


class _GroupRound:
    """adlbq_steal_group_* (the in-library round the bench times) as a round function."""

    def __init__(self, srvs, k):
        self.g = shards.StealGroup(srvs, k, rqcap=1 << 14)

    def __call__(self):
        nd, ns = self.g.round()
        assert self.g.check() == (0, 0)
        return shards.StealResult(self.g.responses(), nd, ns, {})


def _run(S, n_units, R, seed, k, path="host", **kw):
    ws, orcs, resps = build_case(S, n_units, R, seed, **kw)
    srvs = [Server(w.user_types, w.num_app_ranks, S, s, max_units=w.n_units) for s, w in enumerate(ws)]
    grp = None
    try:
        if path == "group_batch":  # shards in a group before their batches: the first export gathers from them
            grp = _GroupRound(srvs, k)
        for s, (w, srv) in enumerate(zip(ws, srvs)):
            out = synth.split_outputs(replay.replay(srv, synth.workload_trace(w)))
            np.testing.assert_array_equal(np.asarray(out[w.n_units:], np.int32), resps[s])
        if path == "group":
            grp = _GroupRound(srvs, k)
        if grp is not None:
            got = rounds(grp)
        else:
            got = rounds(lambda: shards.steal_round_local(srvs, k=k))
        exp = oracle.serial_steal_round(orcs, ws[0].num_app_ranks)
        assert exp.shape[0] > 0
        np.testing.assert_array_equal(got, exp)
        rng = np.random.default_rng(seed)
        for s, (w, srv) in enumerate(zip(ws, srvs)):
            q, hi = srv.qmstat_row()
            oq, ohi = orcs[s].qmrow()
            assert q == oq and hi.tolist() == ohi.tolist()
            # the round answered every SS_RFR the parks sent: the serial model
            # receives each SS_RFR_RESP (adlb.c:1877-1878) as RFRDONE
            rfr = [[synth.OP_RFRDONE, int(r[11]), int(rk)] for r, rk in zip(resps[s], w.r_rank)
                   if r[0] == 0 and r[11] >= 0]
            if rfr:
                orcs[s].replay(np.asarray(rfr, np.int32).ravel())
            tv = synth.type_vectors(rng, w.user_types, 256)
            tr = np.concatenate([synth.simple_events(synth.OP_INFO),
                                 synth.reserve_events(np.arange(256) * S + s, tv, np.zeros(256, np.uint8)),
                                 synth.simple_events(synth.OP_INFO)])
            np.testing.assert_array_equal(replay.replay(srv, tr), orcs[s].replay(tr))
            # parks after the round: their RFR donors (resp[11]) and check_remote
            # see no RFR outstanding from before the round
            tv = synth.type_vectors(rng, w.user_types, 64)
            tr = np.concatenate([synth.reserve_events(np.arange(64) * S + s, tv, np.ones(64, np.uint8)),
                                 synth.simple_events(synth.OP_CHECKREM), synth.simple_events(synth.OP_INFO)])
            np.testing.assert_array_equal(replay.replay(srv, tr), orcs[s].replay(tr))
    finally:
        if grp is not None:
            grp.g.close()
        for srv in srvs:
            srv.close()


# group_batch: the group's first export reads the last Reserve batch's candidate lists (k_export_after)
PATHS = ["host", "group", "group_batch"]


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("S,k", [(2, 4096), (3, 4096), (4, 3)])
def test_steal_round_vs_oracle(gpu_available, S, k, path):
    _run(S, n_units=3000, R=512, seed=40 + S, k=k, path=path)


@pytest.mark.parametrize("path", PATHS)
def test_steal_round_ties_small_k(gpu_available, path):
    _run(3, n_units=2000, R=512, seed=47, k=2, path=path, prio_hi=4)


@pytest.mark.parametrize("path", PATHS)
def test_steal_round_config3_medium(gpu_available, path):
    """Config 3 shape at reduced size: 10% of Reserves have no local type."""
    _run(4, n_units=50_000, R=2048, seed=3, k=1024, path=path, p_remote=0.1, prio_hi=1024)


def test_steal_export_matches_scan(gpu_available):
    """The export is the top k by (prio desc, wqseqno asc) of each type's
    available untargeted units, and leaves the queue unchanged (a Reserve batch
    after it answers as the oracle does)."""
    w = synth.config2(n_units=20_000, n_reserves=1024, seed=48, prio_hi=64)
    w.u_target[::17] = 3
    with Server(w.user_types, w.num_app_ranks, max_units=w.n_units) as srv:
        srv.put_batch(np.stack([w.u_type, w.u_prio, w.u_answer, w.u_target, w.u_len,
                                np.full(w.n_units, -1), np.zeros(w.n_units), np.full(w.n_units, -1),
                                np.full(w.n_units, -1)], axis=1).astype(np.int32))
        recs, nrec, navail = srv.steal_export(700)
        seq = np.arange(1, w.n_units + 1)
        for t in range(w.user_types.size):
            idx = np.nonzero((w.u_type == t) & (w.u_target < 0))[0]
            idx = idx[np.lexsort((seq[idx], -w.u_prio[idx]))]
            assert navail[t] == idx.size and nrec[t] == min(700, idx.size)
            np.testing.assert_array_equal(recs[t, :nrec[t], 0], w.u_prio[idx[:nrec[t]]])
            np.testing.assert_array_equal(recs[t, :nrec[t], 1], seq[idx[:nrec[t]]])
        o = oracle.Oracle("own")
        o.init(w.user_types, w.num_app_ranks)
        o.replay(synth.put_events(w))
        tr = synth.reserve_events(w.r_rank, w.r_types, w.r_hang)
        np.testing.assert_array_equal(replay.replay(srv, tr), o.replay(tr))


def test_grant_and_rq_delete_batches(gpu_available):
    """The synchronous donor / requester entry points: a granted unit is pinned
    (a Reserve no longer sees it, SS_UNRESERVE by the grantee frees it), a
    second grant of it fails; deleting a parked rqseqno twice finds it once."""
    with Server([0, 1], 16, 2, 0, max_units=64) as srv:
        srv.put(0, 10)                                   # wqseqno 1
        srv.put(1, 20)                                   # wqseqno 2
        assert srv.grant_batch([[5, 2], [6, 2], [7, 99]]).tolist() == [1, 0, 0]
        r = srv.reserve(3, [1])                          # type 1: only wqseqno 2, pinned for rank 5
        assert r[0] == 0 and r[10] == 1                  # parked, rqseqno 1
        assert srv.rq_export()[:, :2].tolist() == [[1, 3]]
        assert srv.rq_delete_batch([1, 1, 7]).tolist() == [1, 0, 0]
        assert srv.info()[2] == 0
        assert srv.unreserve(5, 2) == 1
        assert srv.reserve(4, [1])[5] == 2
