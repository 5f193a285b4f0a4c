"""Robustness of the HIP path through the C ABI (failures are loud, growth is bounded).

* an in-launch candidate sort whose wait gives up (k_rank) fails the batch:
  ADLBQ_ERR_DEVICE from the synchronous entry point, ADLB_ERROR in every reply
  of the device entry point, and the queues are left as they were -- never a
  silent wrong match (the sequential handlers of adlb.c:1199-1317 cannot
  half-fail either);
* rq slots are reclaimed: the reference frees every rq node at rq_delete
  (xq.c:379); here dead slots are compacted away (k_rq_reclaim) before the rq
  would grow, so a server that parks and serves Reserves for its whole run
  keeps a bounded rq -- with rqseqnos, FIFO order and every reply as the
  oracle's -- and next_rqseqno stops at the int range with ADLBQ_ERR_NOMEM
  instead of wrapping;
"""
import numpy as np
import pytest

import oracle
from adlb_amd import replay, synth
from adlb_amd._lib import AdlbqError
from adlb_amd.server import Server

pytestmark = pytest.mark.gpu


def _units9(w):
    n = w.n_units
    return np.stack([w.u_type, w.u_prio, w.u_answer, w.u_target, w.u_len, np.full(n, -1), np.zeros(n),
                     np.full(n, -1), np.full(n, -1)], axis=1).astype(np.int32)


def _reqs18(w):
    r = np.empty((w.n_reserves, 18), np.int32)
    r[:, 0], r[:, 1], r[:, 2:] = w.r_rank, w.r_hang, w.r_types
    return r


def test_sort_wait_failure_is_an_error(gpu_available):
    import torch
    w = synth.config2(n_units=20_000, n_reserves=1024, seed=301)
    reqs = _reqs18(w)
    with Server(w.user_types, w.num_app_ranks, max_units=w.n_units) as s:
        s.put_batch(_units9(w))
        s.set_param("sort_fail_test", 1)
        with pytest.raises(AdlbqError, match="rc=-6"):
            s.reserve_batch(reqs)
        d_reqs = torch.from_numpy(reqs).cuda()
        d_resp = torch.full((w.n_reserves, 12), 7, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        s.reserve_batch_device(w.n_reserves, d_reqs.data_ptr(), d_resp.data_ptr())
        s.sync()
        resp = d_resp.cpu().numpy()
        assert (resp[:, 0] == -1).all() and (resp[:, 1:10] == 0).all() and (resp[:, 10:] == -1).all()
        s.set_param("sort_fail_test", 0)
        assert s.stat("batch_failed") == 2
        assert s.info()[2] == 0                 # nothing parked
        # nothing was pinned or parked: the same batch now answers as the oracle does
        got = s.reserve_batch(reqs)
    o = oracle.Oracle("own")
    o.init(w.user_types, w.num_app_ranks)
    o.replay(synth.put_events(w))
    exp = synth.split_outputs(o.replay(synth.reserve_events(w.r_rank, w.r_types, w.r_hang)))
    np.testing.assert_array_equal(got, np.asarray(exp, np.int32))


def _put_events(rng, n, types, prio_hi=8):
    ev = np.empty((n, 10), np.int32)
    ev[:, 0] = synth.OP_PUT
    ev[:, 1] = rng.choice(types, n)
    ev[:, 2] = rng.integers(0, prio_hi, n)
    ev[:, 3] = rng.integers(0, 64, n)
    ev[:, 4] = -1
    ev[:, 5] = 8
    ev[:, 6], ev[:, 7], ev[:, 8], ev[:, 9] = -1, 0, -1, -1
    return ev.ravel()


def _stream(seed, rounds, n_res, n_put, ut, A):
    """Rounds of hanging Reserves that park (the queue is empty or short),
    then Puts that answer most of them (put-side FIFO match, xq.c:388-405);
    some Reserves stay parked for many rounds."""
    rng = np.random.default_rng(seed)
    parts = []
    for _ in range(rounds):
        tv = synth.type_vectors(rng, ut, n_res)
        parts.append(synth.reserve_events(rng.integers(0, A, n_res), tv, np.ones(n_res, np.uint8)))
        parts.append(_put_events(rng, n_put, ut))
    return np.concatenate(parts)


def test_rq_slots_reclaimed_vs_oracle(gpu_available):
    ut, A = np.arange(3, dtype=np.int32), 4096
    # batches of 512: the rq headroom a host may run ahead by (NSNAP batches) stays far below the parks
    tr = _stream(11, rounds=160, n_res=512, n_put=500, ut=ut, A=A)
    with Server(ut, A, max_units=1 << 16) as s:
        got = replay.replay(s, tr)
        parks = s.stat("rq_next")
        assert parks > 40_000, parks
        assert s.stat("rq_reclaims") > 0
        assert s.stat("rq_cap") < parks // 2, (s.stat("rq_cap"), parks)   # without reclaim: >= parks
        assert s.stat("rq_slots") <= s.stat("rq_cap")
    o = oracle.Oracle("own")
    o.init(ut, A)
    np.testing.assert_array_equal(got, o.replay(tr))


def test_rqseqno_overflow_is_nomem(gpu_available):
    ut = np.arange(2, dtype=np.int32)
    with Server(ut, 64, max_units=1024) as s:
        s.set_param("rq_next", (1 << 31) - 1 - 100)
        r = s.reserve_batch([[3, 1, 0] + [-2] * 15] * 50)     # 50 parks: rqseqnos up to INT_MAX - 50
        assert (r[:, 0] == 0).all() and r[-1, 10] == (1 << 31) - 1 - 50
        with pytest.raises(AdlbqError, match="rc=-3"):
            s.reserve_batch([[4, 1, 1] + [-2] * 15] * 64)     # could take rqseqnos past INT_MAX
        assert s.stat("rq_next") == (1 << 31) - 1 - 50


@pytest.mark.parametrize("path,n_units,n_res", [("small", 9_000, 700), ("one", 30_000, 1)])
def test_choice_outside_page_list_is_an_error(gpu_available, path, n_units, n_res):
    """The round-5 fault: a choice of the one-workgroup paths
    (k_reserve_small, k_reserve_one) whose bucket position lies past the open
    bucket's page list.  It is driven directly ("bound_inject" tells the next
    choice such a position): the batch is answered ADLB_ERROR and counted
    (stat bound_faults), the synchronous entry returns ADLBQ_ERR_DEVICE, nothing
    is pinned or parked, and the same batch then answers as the oracle does."""
    w = synth.config2(n_units=n_units, n_reserves=n_res, seed=303)
    reqs = _reqs18(w)
    with Server(w.user_types, w.num_app_ranks, max_units=w.n_units) as s:
        s.put_batch(_units9(w))
        s.set_param("bound_inject", 1)
        with pytest.raises(AdlbqError, match="rc=-6"):
            s.reserve_batch(reqs)
        assert s.stat("bound_faults") == 1
        assert s.stat("batch_failed") == 1
        assert s.info()[2] == 0                 # nothing parked
        assert s.stat(path + "_batches") == 1   # the path under test took the batch
        got = s.reserve_batch(reqs)             # the flag is one-shot: the same batch, now correct
        assert s.stat("bound_faults") == 1
    o = oracle.Oracle("own")
    o.init(w.user_types, w.num_app_ranks)
    o.replay(synth.put_events(w))
    exp = synth.split_outputs(o.replay(synth.reserve_events(w.r_rank, w.r_types, w.r_hang)))
    np.testing.assert_array_equal(got, np.asarray(exp, np.int32))
