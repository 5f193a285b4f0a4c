"""Config 5 at its SURVEY §8(d) shape (oracle/gen_c5.c): S server shards'
tsp.c-style streams with a qmstat snapshot and a steal round every 10^4
events, replayed through the engine ABI by adlbsrv_replay_rounds (device-side
batches between rounds, one steal-group round at each marker).  Every event's
output and every steal must equal the oracle's, which runs the same rounds
one SS_RFR exchange at a time (adlb.c:1802-1933)."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def _check(S, A, n_events, k, q0, seed, closed=False):
    from adlb_amd import replay
    from adlb_amd.server import Server
    d = oracle.gen_config5(n_shards=S, n_ranks=A, n_events=n_events, round_every=10_000, k=k, q0=q0, seed=seed)
    assert d["rounds"] >= n_events // 12_000 and d["steals"].shape[0] > 0, (d["rounds"], d["steals"].shape)
    srvs = [Server(d["user_types"], A, S, s, max_units=1 << 16) for s in range(S)]
    st = {}
    try:
        got, steals, _, _ = replay.replay_rounds(srvs, d["traces"], k=k, rqcap=A, closed=closed, stats=st)
    finally:
        for s in srvs:
            s.close()
    for s in range(S):
        e = d["outputs"][s]
        assert got[s].size == e.size, (s, got[s].size, e.size)
        bad = np.nonzero(got[s] != e)[0]
        assert bad.size == 0, f"shard {s}: first mismatch at output int {bad[0]}: {got[s][bad[0]]} vs {e[bad[0]]}"
    key = lambda a: a[np.lexsort((a[:, 1], a[:, 0]))] if a.size else a
    # the rounds' steals, round by round in serial order; the engine reports them per round too
    np.testing.assert_array_equal(np.sort(steals.view([("", steals.dtype)] * 15), axis=0),
                                  np.sort(d["steals"].view([("", steals.dtype)] * 15), axis=0))
    if closed:  # every Get's wqseqno came from a landed reply, and it is the recorded one
        assert st["wqseqno_mismatch"] == 0, st
    d["closed_stats"] = st
    return d


def test_config5_shape_small_vs_oracle(gpu_available):
    d = _check(S=4, A=1024, n_events=300_000, k=64, q0=128, seed=3)
    assert d["stopped"] >= 0


def test_config5_shape_rounds_that_stop_vs_oracle(gpu_available):
    """An export depth of 4: rounds stop at the first Reserve that would need
    a unit past a shard's exported top 4 (adlbq_steal.hip merge_views), and the
    generator's serial rounds stop at the same Reserve."""
    d = _check(S=8, A=2048, n_events=200_000, k=4, q0=128, seed=4)
    assert d["stopped"] > 0, d["stopped"]


def test_config5_closed_loop_vs_oracle(gpu_available):
    """Closed loop (adlbsrv_replay_rounds2): a shard issues each Get only after
    the reply it depends on -- its TA_RESERVE_RESP, the put-side match of its
    parked Reserve, or the steal round's answer -- has landed in mapped host
    memory, and takes the wqseqno from that reply (tsp.c:157-162).  Outputs and
    steals equal the oracle's, and every reply's wqseqno is the recorded Get's."""
    d = _check(S=4, A=1024, n_events=200_000, k=64, q0=128, seed=5, closed=True)
    assert d["closed_stats"]["get_calls_waited"] >= 0
