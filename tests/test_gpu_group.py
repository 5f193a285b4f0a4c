"""adlbq_reserve_group_device (include/adlbq.h): the Reserve batches of several
local server shards as one launch per pipeline kernel (grid.y = shard) give
each shard the answers of its own sequential run -- the oracle's
-- batch after batch, in the mixes a process's shards can be in: shards that
group, a shard of another type-count class (its own launches), a shard with
targeted units (it leaves the group at the targeted index), a shard with
grouping turned off, and an empty batch.
"""
import numpy as np
import pytest

import oracle
from adlb_amd import synth

pytestmark = pytest.mark.gpu


def _units(w):
    n = w.n_units
    return np.stack([w.u_type, w.u_prio, w.u_answer, w.u_target, w.u_len, np.full(n, -1), np.zeros(n),
                     np.full(n, -1), np.full(n, -1)], axis=1).astype(np.int32)


def _shards(S, n_units, R, seed):
    """(workload, shard index, params) per local shard of an S-shard queue."""
    out = []
    for s in range(S):
        T = 6 if s == 3 else 4          # shard 3: the 8-wide kernels, a group of its own
        w = synth.config3_shard(s, S, n_units, T, R, seed=seed + s, prio_hi=64, p_remote=0.1)
        params = {}
        if s == 4:                      # targeted units: the batch leaves the group at the targeted index
            rng = np.random.default_rng(seed + 99)
            tg = rng.random(n_units) < 0.05
            w.u_target[tg] = (rng.integers(0, R, int(tg.sum())) * S + s).astype(np.int32)
        if s == 5:
            params["group_launch"] = 0  # launched alone
        out.append((w, s, params))
    return out


def _oracle_resps(w, S, s):
    o = oracle.Oracle("own", private=True)
    o.init(w.user_types, w.num_app_ranks, S, s)
    out = synth.split_outputs(o.replay(synth.workload_trace(w)))
    return np.asarray(out[w.n_units:], dtype=np.int32)


@pytest.mark.parametrize("params", [{}, {"rank_in_select": 0}], ids=["default", "rank_in_k_rank"])
def test_group_matches_sequential(gpu_available, params):
    import torch
    from adlb_amd.server import ReserveGroup, Server

    S, N, R, nb = 7, 30_000, 3072, 3
    specs = _shards(S, N, R, seed=41)
    exp = [_oracle_resps(w, S, s) for w, s, _ in specs]
    srvs, streams, d_req, d_resp = [], [], [], []
    try:
        for w, s, p in specs:
            srv = Server(w.user_types, w.num_app_ranks, S, s, max_units=N)
            srvs.append(srv)
            for k, v in {**params, **p}.items():
                srv.set_param(k, v)
            st = torch.cuda.Stream()
            srv.set_stream(st.cuda_stream)
            streams.append(st)
            srv.put_batch(_units(w))
            reqs = np.concatenate([w.r_rank[:, None], w.r_hang[:, None].astype(np.int32), w.r_types],
                                  axis=1).astype(np.int32)
            d_req.append(torch.from_numpy(reqs).cuda())
            d_resp.append(torch.full((R, 12), -7, dtype=torch.int32, device="cuda"))
        torch.cuda.synchronize()
        grp = ReserveGroup(srvs)
        for b in range(nb):
            lo, hi = b * R // nb, (b + 1) * R // nb
            counts = [hi - lo] * S
            if b == 1:
                counts[6] = 0  # an empty batch in the group; shard 6 runs this one alone after it
            grp.reserve_device(counts, [d.data_ptr() + lo * 18 * 4 for d in d_req],
                               [d.data_ptr() + lo * 12 * 4 for d in d_resp])
            if b == 1:
                srvs[6].reserve_batch_device(hi - lo, d_req[6].data_ptr() + lo * 18 * 4,
                                             d_resp[6].data_ptr() + lo * 12 * 4)
        torch.cuda.synchronize()
        for j, (w, s, _) in enumerate(specs):
            got = d_resp[j].cpu().numpy()
            assert np.array_equal(got[:, :10], exp[j][:, :10]), f"shard {s}"
        # the last batch again after unreserving it: same answers (queues restored, hints landed)
        lo = (nb - 1) * R // nb
        grp.unreserve_resp_device([R - lo] * S, [d.data_ptr() + lo * 18 * 4 for d in d_req],
                                  [d.data_ptr() + lo * 12 * 4 for d in d_resp])
        before = [d[lo:].cpu().numpy().copy() for d in d_resp]
        torch.cuda.synchronize()
        grp.reserve_device([R - lo] * S, [d.data_ptr() + lo * 18 * 4 for d in d_req],
                           [d.data_ptr() + lo * 12 * 4 for d in d_resp])
        torch.cuda.synchronize()
        for j in range(S):  # parked Reserves park again (new rq entries): compare the matched rows whole
            again = d_resp[j][lo:].cpu().numpy()
            assert np.array_equal(again[:, 0], before[j][:, 0]), f"shard {j} again"
            m = before[j][:, 0] == 1
            assert m.any() and np.array_equal(again[m, :10], before[j][m, :10]), f"shard {j} again"
    finally:
        torch.cuda.synchronize()
        for srv in srvs:
            srv.close()


def test_group_rejects_bad_arguments(gpu_available):
    import torch
    from adlb_amd import _lib
    from adlb_amd.server import ReserveGroup, Server

    w = synth.config3_shard(0, 2, 1000, 4, 64, seed=5)
    with Server(w.user_types, w.num_app_ranks, 2, 0, max_units=1000) as a:
        d = torch.zeros((64, 18), dtype=torch.int32, device="cuda")
        r = torch.zeros((64, 12), dtype=torch.int32, device="cuda")
        with pytest.raises(_lib.AdlbqError):
            ReserveGroup([a, a]).reserve_device([64, 64], [d.data_ptr()] * 2, [r.data_ptr()] * 2)
        with pytest.raises(_lib.AdlbqError):
            ReserveGroup([a]).reserve_device([64], [0], [r.data_ptr()])
        ReserveGroup([a]).reserve_device([0], [0], [0])  # nothing to do


def test_group_many_small_shards(gpu_available):
    """40 small shards in one group (the argument tables outgrow their first
    allocation; grid.y = 40): every shard's answers equal its own sequential
    run's, over two batches."""
    import torch
    from adlb_amd.server import ReserveGroup, Server

    S, N, R = 40, 2_000, 512
    specs = [(synth.config3_shard(s, S, N, 4, R, seed=300 + s, prio_hi=32, p_remote=0.1), s) for s in range(S)]
    exp = [_oracle_resps(w, S, s) for w, s in specs]
    srvs, d_req, d_resp = [], [], []
    st = torch.cuda.Stream()
    try:
        for w, s in specs:
            srv = Server(w.user_types, w.num_app_ranks, S, s, max_units=N)
            srvs.append(srv)
            srv.set_stream(st.cuda_stream)  # one shared stream, as the bench runs them
            srv.put_batch(_units(w))
            reqs = np.concatenate([w.r_rank[:, None], w.r_hang[:, None].astype(np.int32), w.r_types],
                                  axis=1).astype(np.int32)
            d_req.append(torch.from_numpy(reqs).cuda())
            d_resp.append(torch.full((R, 12), -7, dtype=torch.int32, device="cuda"))
        torch.cuda.synchronize()
        grp = ReserveGroup(srvs)
        for lo, hi in ((0, R // 2), (R // 2, R)):
            grp.reserve_device([hi - lo] * S, [d.data_ptr() + lo * 18 * 4 for d in d_req],
                               [d.data_ptr() + lo * 12 * 4 for d in d_resp])
        torch.cuda.synchronize()
        for j, (w, s) in enumerate(specs):
            assert np.array_equal(d_resp[j].cpu().numpy()[:, :10], exp[j][:, :10]), f"shard {s}"
    finally:
        torch.cuda.synchronize()
        for srv in srvs:
            srv.close()
