"""Config 3's cross-process steal round on HIP shards.

Two processes (world size 2, gloo over 127.0.0.1) share the one GPU; each
holds two of the four server shards as HIP handles in one StealGroup, the way
a GPU process holds its group of servers.  Every round exports each process's
blob (adlbq_steal_group_export_host), all-gathers the blobs across the
processes and settles the same merge everywhere (adlbq_steal_group_settle_host,
nproc = 2): each process pins what its donors granted and answers its own
parked Reserves.  The settlements must equal oracle.serial_steal_round (the
SS_RFR / SS_RFR_RESP exchanges of adlb.c:1802-1933 serialised) at the
test_steal_round_config3_medium shape, and afterwards every shard must answer
a further Reserve batch as its oracle does.
"""
import os
import socket
import traceback

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

S, N_UNITS, R, SEED, K = 4, 50_000, 2048, 3, 1024
KW = dict(p_remote=0.1, prio_hi=1024)


def _worker(rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist

        import oracle
        from adlb_amd import replay, shards, synth
        from adlb_amd.server import Server
        from steal_case import build_case

        torch.cuda.set_device(0)
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ws, orcs, resps = build_case(S, N_UNITS, R, SEED, **KW)
        mine = [s for s in range(S) if s * world // S == rank]      # contiguous shard groups
        srvs = {s: Server(ws[s].user_types, ws[s].num_app_ranks, S, s, max_units=ws[s].n_units) for s in mine}
        grp = shards.StealGroup([srvs[s] for s in mine], K, rqcap=1 << 14)
        try:
            for s in mine:
                out = synth.split_outputs(replay.replay(srvs[s], synth.workload_trace(ws[s])))
                np.testing.assert_array_equal(np.asarray(out[ws[s].n_units:], np.int32), resps[s])
            got, nrounds = [], 0
            while True:
                nd, ns = grp.round()
                assert grp.check() == (0, 0)
                got.append(grp.responses())
                nrounds += 1
                if ns == 0:
                    break
            got = np.concatenate(got)
            exp = oracle.serial_steal_round(orcs, ws[0].num_app_ranks)
            assert exp.shape[0] > 0
            e = exp[np.isin(exp[:, 0], mine)]
            assert e.shape[0] > 0, "no settlement lands on this process's shards"
            np.testing.assert_array_equal(got[np.lexsort((got[:, 1], got[:, 0]))],
                                          e[np.lexsort((e[:, 1], e[:, 0]))])
            rng = np.random.default_rng(SEED)
            for s in mine:
                srv, o, w = srvs[s], orcs[s], ws[s]
                qn, hi = srv.qmstat_row()
                oq, ohi = o.qmrow()
                assert qn == oq and hi.tolist() == ohi.tolist()
                rfr = [[synth.OP_RFRDONE, int(r[11]), int(rk)] for r, rk in zip(resps[s], w.r_rank)
                       if r[0] == 0 and r[11] >= 0]
                if rfr:
                    o.replay(np.asarray(rfr, np.int32).ravel())
                tv = synth.type_vectors(rng, w.user_types, 256)
                tr = np.concatenate([synth.simple_events(synth.OP_INFO),
                                     synth.reserve_events(np.arange(256) * S + s, tv, np.zeros(256, np.uint8)),
                                     synth.simple_events(synth.OP_INFO)])
                np.testing.assert_array_equal(replay.replay(srv, tr), o.replay(tr))
            q.put((rank, "ok", int(got.shape[0]), nrounds))
        finally:
            grp.close()
            for srv in srvs.values():
                srv.close()
            dist.destroy_process_group()
    except BaseException:
        q.put((rank, traceback.format_exc(), 0, 0))
        raise


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def test_steal_group_two_processes_vs_oracle(gpu_available):
    import multiprocessing as mp
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r = q.get(timeout=100)
            res[r[0]] = r
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert res[r][1] == "ok", res[r][1]
    assert sum(res[r][2] for r in range(world)) > 0
    assert res[0][3] == res[1][3]          # both processes ran the same rounds


def test_steal_group_device_blobs_two_groups_vs_oracle(gpu_available):
    """The RCCL branch of StealGroup.round without the collective: two
    StealGroups of two HIP shards each (the shards two GPU processes would
    hold) export into adjacent halves of ONE device tensor -- exactly the
    [nproc][blob] layout all_gather_into_tensor delivers -- and each settles
    over it with nproc = 2 (adlbq_steal_group_export(g, d_blob) ->
    adlbq_steal_group_settle(g, d_all, 2)).  Settlements, qmstat rows and a
    follow-up Reserve batch per shard must equal oracle.serial_steal_round and
    the oracle shards (adlb.c:1802-1933, 3536-3579)."""
    import torch

    import oracle
    from adlb_amd import replay, shards, synth
    from adlb_amd.server import Server
    from steal_case import build_case

    ws, orcs, resps = build_case(S, N_UNITS, R, SEED, **KW)
    groups_of = [[0, 1], [2, 3]]
    srvs = {s: Server(ws[s].user_types, ws[s].num_app_ranks, S, s, max_units=ws[s].n_units) for s in range(S)}
    grps = [shards.StealGroup([srvs[s] for s in m], K, rqcap=1 << 14) for m in groups_of]
    try:
        for s in range(S):
            out = synth.split_outputs(replay.replay(srvs[s], synth.workload_trace(ws[s])))
            np.testing.assert_array_equal(np.asarray(out[ws[s].n_units:], np.int32), resps[s])
        bi = grps[0].blob_ints
        assert grps[1].blob_ints == bi
        d_all = torch.full((2 * bi,), -7, dtype=torch.int32, device="cuda:0")
        got = [[] for _ in grps]
        nrounds = 0
        while True:
            for p, g in enumerate(grps):       # each "process" exports into its slot
                g.export_device(d_all.data_ptr() + p * bi * 4)
            for s in srvs.values():            # as StealGroup.round does before the collective
                s.sync()
            res = [g.settle_device(d_all.data_ptr(), 2) for g in grps]
            assert res[0] == res[1], "both processes must decide and settle the same round"
            for p, g in enumerate(grps):
                assert g.check() == (0, 0)
                got[p].append(g.responses())
            nrounds += 1
            if res[0][1] == 0:
                break
        assert nrounds >= 2
        exp = oracle.serial_steal_round(orcs, ws[0].num_app_ranks)
        assert exp.shape[0] > 0
        for p, m in enumerate(groups_of):
            gp = np.concatenate(got[p])
            e = exp[np.isin(exp[:, 0], m)]
            assert e.shape[0] > 0, f"no settlement lands on group {p}"
            np.testing.assert_array_equal(gp[np.lexsort((gp[:, 1], gp[:, 0]))], e[np.lexsort((e[:, 1], e[:, 0]))])
        rng = np.random.default_rng(SEED)
        for s in range(S):
            srv, o, w = srvs[s], orcs[s], ws[s]
            qn, hi = srv.qmstat_row()
            oq, ohi = o.qmrow()
            assert qn == oq and hi.tolist() == ohi.tolist()
            rfr = [[synth.OP_RFRDONE, int(r[11]), int(rk)] for r, rk in zip(resps[s], w.r_rank)
                   if r[0] == 0 and r[11] >= 0]
            if rfr:
                o.replay(np.asarray(rfr, np.int32).ravel())
            tv = synth.type_vectors(rng, w.user_types, 256)
            tr = np.concatenate([synth.simple_events(synth.OP_INFO),
                                 synth.reserve_events(np.arange(256) * S + s, tv, np.zeros(256, np.uint8)),
                                 synth.simple_events(synth.OP_INFO)])
            np.testing.assert_array_equal(replay.replay(srv, tr), o.replay(tr))
    finally:
        for g in grps:
            g.close()
        for srv in srvs.values():
            srv.close()
