"""Multi-shard host logic on CPU: world_size-2 gloo process groups.

* exchange_qmstat: every shard ends with the table the reference's qmstat ring
  converges to (row i = server i's update_local_state), and donor selection
  (check_remote_work_for_queued_apps, adlb.c:3536-3579) run on that table
  picks the other shard -- checked with the oracle as the shard backend;
* reduce_step_timing: max of elapsed, sum of matched over ranks.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle
from adlb_amd import shards, synth

A = 8  # app ranks; server world ranks are A + shard index (adlb.c:246-258)
UT = [0, 1, 2]


class OracleShard:
    """Duck-typed stand-in for adlb_amd.server.Server backed by the CPU oracle."""

    def __init__(self, idx, nshards):
        self.o = oracle.Oracle("own")
        self.o.init(UT, A, nshards, idx)
        self.T = len(UT)
        self.my_server_idx = idx

    def run(self, ev):
        return synth.split_outputs(self.o.replay(ev))

    def qmstat_row(self):
        r = self.run(synth.simple_events(oracle.OP_QMROW))[0]
        return r[0], np.asarray(r[1:1 + self.T], np.int32)

    def set_qmstat_row(self, idx, qlen, nbytes, hi):
        self.run(synth.simple_events(oracle.OP_SETROW, idx, qlen, int(nbytes), *[int(x) for x in hi]))

    def check_remote(self):
        r = self.run(synth.simple_events(oracle.OP_CHECKREM))[0]  # {k, k x (rqseqno, rank, donor)}
        return np.asarray(r[1:1 + 3 * r[0]], np.int32).reshape(-1, 3)


def _put(s, t, prio, n):
    ev = np.concatenate([synth.simple_events(oracle.OP_PUT, t, prio, 0, -1, 8, -1, 0, -1, -1) for _ in range(n)])
    s.run(ev)


class GpuShard:
    """The HIP server handle (adlb_amd.server.Server) as a shard."""

    def __init__(self, idx, nshards):
        from adlb_amd.server import Server
        self.s = Server(UT, A, nshards, idx)
        self.T = len(UT)
        self.my_server_idx = idx

    def run(self, ev):
        from adlb_amd import replay
        return synth.split_outputs(replay.replay(self.s, ev))

    def qmstat_row(self):
        return self.s.qmstat_row()

    def set_qmstat_row(self, idx, qlen, nbytes, hi):
        self.s.set_qmstat_row(idx, qlen, nbytes, hi)

    def check_remote(self):
        return self.s.check_remote()


def _worker(rank, world, port, q, kind="oracle"):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s = OracleShard(rank, world) if kind == "oracle" else GpuShard(rank, world)
        if rank == 0:
            _put(s, 0, 5, 3)                 # shard 0 holds type 0 only
        else:
            _put(s, 1, 9, 2)                 # shard 1 holds types 1 and 0
            _put(s, 0, 7, 1)
        # app rank 3 asks shard 0 for type 1 and parks (no local type-1 work,
        # and the table is still empty, so no RFR goes out yet)
        tv = [1] + [-2] * 15
        resp = s.run(synth.reserve_events([3], [tv], [1]))[0] if rank == 0 else None
        table = shards.exchange_qmstat(s)
        rem = s.check_remote()
        el, matched = shards.reduce_step_timing(0.5 + rank, 10 * (rank + 1))
        q.put((rank, table.tolist(), rem.tolist(), resp, el, matched))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _run_pair(kind):
    if not oracle.available("own"):
        oracle.build()
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, kind)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r = q.get(timeout=60)
        got[r[0]] = r
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    t0, t1 = np.array(got[0][1]), np.array(got[1][1])
    assert np.array_equal(t0, t1)
    # rows: {qlen, nbytes, hi[0], hi[1], hi[2]}
    assert t0[0, 0] == 3 and list(t0[0, 2:]) == [5, -999999999, -999999999]
    assert t0[1, 0] == 3 and list(t0[1, 2:]) == [7, 9, -999999999]
    resp = got[0][3]
    assert resp[0] == 0 and resp[11] == -1          # parked, no donor known yet
    rqseqno = resp[10]
    # after the exchange shard 0 sends an RFR for the parked request to shard 1
    assert got[0][2] == [[rqseqno, 3, A + 1]]
    assert got[1][2] == []
    for r in range(world):
        assert got[r][4] == 1.5 and got[r][5] == 30


def test_exchange_qmstat_and_donor_gloo():
    _run_pair("oracle")


@pytest.mark.gpu
def test_exchange_qmstat_and_donor_gpu_shards(gpu_available):
    """Two HIP server shards on the one GPU, rows exchanged over gloo: same table
    and the same RFR decision as the oracle shards."""
    _run_pair("gpu")


@pytest.mark.parametrize("rank", [0, 1, 7])
def test_shard_seed_distinct(rank):
    assert shards.shard_seed(2, rank) == 2 + 1000 * rank
    assert len({shards.shard_seed(2, r) for r in range(8)}) == 8
