"""One ADLB server shard per GPU process.

The reference shards its queues by server rank: each server's wq/rq/tq are
process globals (src/xq.c:11-15) and matching never reads another server's
queue.  Here one process per GPU owns one server handle; the only cross-shard
traffic of the hot path is the qmstat status table, which the reference passes
hop by hop around a ring of servers every ~0.1 s (src/adlb.c:1705-1757,
3178-3220).  `exchange_qmstat` replaces that ring with one all-gather over the
process group (RCCL on GPU ranks, gloo on CPU), after which every shard holds
the same table the ring converges to: row i = server i's update_local_state
output (adlb.c:3581-3593).  Donor selection (find_cand_rank_with_worktype,
adlb.c:3487-3534) then runs on each shard against that table
(Server.check_remote).

The steal round (`steal_round`) replaces the SS_RFR /
SS_RFR_RESP round trips (adlb.c:1280-1308, 1802-1933): every shard exports its
top-k available units per type and its parked Reserves, one all-gather moves
them to every process, and every process runs the same deterministic merge
(adlbq_steal_merge in the library: the round trips serialised in (shard,
rqseqno) order against the donors' current heads).  Donors then pin what the
merge granted and requesters answer their apps and drop the rq entries -- no
further exchange, since every process computed the same grants.

`reduce_step_timing` is the bench's max-over-ranks / sum-over-ranks reduction.
"""
from __future__ import annotations

import ctypes
import time
from typing import NamedTuple

import numpy as np

from . import _lib


def shard_seed(base: int, rank: int) -> int:
    """Per-shard workload seed: every shard gets its own queue and Reserve stream."""
    return int(base) + 1000 * int(rank)


def _dev_of(group_backend: str):
    import torch
    return torch.device("cuda", torch.cuda.current_device()) if group_backend == "nccl" else torch.device("cpu")


def exchange_qmstat(srv, group=None) -> np.ndarray:
    """All-gather every shard's qmstat row and install the other shards' rows.

    srv: an object with qmstat_row() -> (qlen, type_hi_prio[T]),
    set_qmstat_row(idx, qlen, nbytes, hi), .T and .my_server_idx (adlb_amd.server.Server).
    Returns the gathered table as int64 [S, 2 + T]: {qlen, nbytes_used, hi[T]}.
    The shard index of rank r is r (one server per process)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    me = dist.get_rank(group)
    if srv.my_server_idx != me:
        raise ValueError(f"shard index {srv.my_server_idx} != process rank {me}")
    qlen, hi = srv.qmstat_row()
    nbytes = int(getattr(srv, "nbytes_used", 0))
    row = np.concatenate([[qlen, nbytes], np.asarray(hi, np.int64)]).astype(np.int64)
    dev = _dev_of(dist.get_backend(group))
    mine = torch.from_numpy(row).to(dev)
    rows = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(rows, mine, group=group)
    table = torch.stack(rows).cpu().numpy()
    for i in range(world):
        if i != me:
            srv.set_qmstat_row(i, int(table[i, 0]), float(table[i, 1]), table[i, 2:].astype(np.int32))
    return table


def reduce_step_timing(elapsed_s: float, matched: int, group=None):
    """(max elapsed over ranks, sum of matched over ranks): the whole-job time
    is the slowest shard's, the work is every shard's."""
    import torch
    import torch.distributed as dist
    dev = _dev_of(dist.get_backend(group))
    t = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    m = torch.tensor([int(matched)], dtype=torch.int64, device=dev)
    dist.all_reduce(m, op=dist.ReduceOp.SUM, group=group)
    return float(t.item()), int(m.item())


# ------------------------------------------------------------------ steal round
class StealResult(NamedTuple):
    resp: np.ndarray   # (m, 15) {shard, rqseqno, rank, TA_RESERVE_RESP[12]} for local requesters
    decided: int       # Reserves the merge decided, all shards
    settled: int       # Reserves it settled (a donor granted a unit), all shards
    grants: dict       # local donor shard -> (n, 2) {rank, wqseqno} it pinned


def steal_merge(user_types, k: int, recs, nrec, navail, reqs19):
    """The merge over S shards (adlbq_steal_merge): recs [S, T, k, 8], nrec [S, T],
    navail [S, T], reqs19 (n, 19) {shard, rqseqno, rank, types[16]} in (shard,
    rqseqno) order -> (out (n, 3) {donor shard, type index, record index} or -1,
    number of requests decided)."""
    lib = _lib.load()
    ut = np.ascontiguousarray(np.asarray(user_types, dtype=np.int32))
    recs = np.ascontiguousarray(np.asarray(recs, dtype=np.int32))
    S, T = recs.shape[0], ut.size
    nrec = np.ascontiguousarray(np.asarray(nrec, dtype=np.int32).reshape(S, T))
    navail = np.ascontiguousarray(np.asarray(navail, dtype=np.int64).reshape(S, T))
    q = np.ascontiguousarray(np.asarray(reqs19, dtype=np.int32).reshape(-1, 19))
    out = np.empty((q.shape[0], 3), dtype=np.int32)
    nd = ctypes.c_int()
    _lib.check(lib.adlbq_steal_merge(S, T, ut.ctypes.data, int(k), recs.ctypes.data, nrec.ctypes.data,
                                     navail.ctypes.data, q.shape[0], q.ctypes.data, out.ctypes.data,
                                     ctypes.byref(nd)), "adlbq_steal_merge")
    return out, nd.value


def _sort_reqs(reqs19: np.ndarray) -> np.ndarray:
    if reqs19.shape[0] == 0:
        return reqs19
    return reqs19[np.lexsort((reqs19[:, 1], reqs19[:, 0]))]


def _tick(timing, key, t0):
    if timing is not None:
        t = time.perf_counter()
        timing[key] = timing.get(key, 0.0) + (t - t0)
        return t
    return t0


def settle(local, num_app_ranks: int, user_types, k: int, recs, nrec, navail, reqs19, timing=None):
    """Run the merge on the gathered exports and apply this process's side of it.

    local: {shard index: server} for the shards this process owns (objects with
    steal_apply and steal_check, e.g. adlb_amd.server.Server).
    Returns a StealResult: the responses for the Reserves of local shards that
    were settled (the reply SS_RFR_RESP sends the app, adlb.c:1885-1898, with
    the donor's world rank), the numbers of Reserves the merge decided and
    settled over all shards (the same on every process), and the units each
    local donor pinned."""
    t0 = time.perf_counter()
    reqs19 = _sort_reqs(np.asarray(reqs19, dtype=np.int32).reshape(-1, 19))
    out, nd = steal_merge(user_types, k, recs, nrec, navail, reqs19)
    t0 = _tick(timing, "merge", t0)
    won = np.nonzero(out[:nd, 0] >= 0)[0]
    d, t, i = out[won, 0], out[won, 1], out[won, 2]
    r = recs[d, t, i]                                  # [m, 8] records of the granted units
    q = reqs19[won]
    grants = {s: np.stack([q[g, 2], r[g, 1]], axis=1).astype(np.int32)
              for s in local for g in [np.nonzero(d == s)[0]] if g.size}
    mine = np.isin(q[:, 0], np.fromiter(local.keys(), dtype=np.int32, count=len(local)))
    resp = np.empty((int(mine.sum()), 15), dtype=np.int32)
    qm, rm, dm = q[mine], r[mine], d[mine]
    resp[:, 0:3] = qm[:, 0:3]
    resp[:, 3] = 1                                     # SUCCESS
    resp[:, 4] = rm[:, 2]                              # work_type
    resp[:, 5] = rm[:, 0]                              # work_prio
    resp[:, 6] = rm[:, 3]                              # work_len
    resp[:, 7] = rm[:, 4]                              # answer_rank
    resp[:, 8] = rm[:, 1]                              # wqseqno
    resp[:, 9] = num_app_ranks + dm                    # donor server's world rank
    resp[:, 10:13] = rm[:, 5:8]                        # common_len, common_server, common_seqno
    resp[:, 13:15] = -1
    empty = np.zeros((0, 2), np.int32)
    for s, srv in local.items():                       # enqueue every shard's side, then check
        srv.steal_apply(grants.get(s, empty), resp[resp[:, 0] == s, 1])
    for s, srv in local.items():
        bg, bd = srv.steal_check()
        if bg or bd:
            raise RuntimeError(f"shard {s}: {bg} granted units no longer available, "
                               f"{bd} settled Reserves no longer parked")
    _tick(timing, "apply", t0)
    return StealResult(resp, nd, int(won.size), grants)


def _export_all(servers, k: int):
    """Every local shard's export: all scans enqueued first (one stream each),
    then collected -> list of (recs, nrec, navail, reqs19)."""
    for srv in servers:
        srv.steal_begin(k)
    out = []
    for srv in servers:
        recs, nrec, navail, rq = srv.steal_collect()
        reqs = np.empty((rq.shape[0], 19), dtype=np.int32)
        reqs[:, 0] = srv.my_server_idx
        reqs[:, 1:] = rq
        out.append((recs, nrec, navail, reqs))
    return out


def steal_round_local(servers, k: int, timing=None):
    """The steal round among shards held by one process (no collective)."""
    t0 = time.perf_counter()
    S = servers[0].num_servers
    T = servers[0].T
    recs = np.zeros((S, T, k, 8), np.int32)
    nrec = np.zeros((S, T), np.int32)
    navail = np.zeros((S, T), np.int64)
    reqs = []
    for srv, (a, b, c, q) in zip(servers, _export_all(servers, k)):
        recs[srv.my_server_idx], nrec[srv.my_server_idx], navail[srv.my_server_idx] = a, b, c
        reqs.append(q)
    _tick(timing, "export", t0)
    local = {srv.my_server_idx: srv for srv in servers}
    return settle(local, servers[0].num_app_ranks, servers[0].user_types, k, recs, nrec, navail,
                  np.concatenate(reqs) if reqs else np.zeros((0, 19), np.int32), timing)


def steal_round(servers, k: int, group=None, timing=None):
    """The steal round across processes: each process holds `servers` (its
    shards); one all-gather of sizes and one of the padded exports (RCCL over
    xGMI on GPU ranks, gloo on CPU), then the same merge everywhere."""
    import torch
    import torch.distributed as dist
    S, T = servers[0].num_servers, servers[0].T
    dev = _dev_of(dist.get_backend(group))
    world = dist.get_world_size(group)
    # one int32 blob per process: per shard [idx, nrec[T], navail lo/hi [2T], recs[T*k*8]], then reqs
    per = 1 + 3 * T + T * k * 8
    t0 = time.perf_counter()
    parts, reqs = [], []
    for srv, (a, b, c, q) in zip(servers, _export_all(servers, k)):
        nav = np.ascontiguousarray(c.astype(np.int64)).view(np.int32)
        parts.append(np.concatenate([[srv.my_server_idx], b, nav, a.ravel()]).astype(np.int32))
        reqs.append(q.ravel())
    blob = np.concatenate([[len(servers)], *parts, *reqs]).astype(np.int32)
    t0 = _tick(timing, "export", t0)
    n = torch.tensor([blob.size], dtype=torch.int64, device=dev)
    sizes = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    cap = int(max(int(x.item()) for x in sizes))
    mine = torch.zeros(cap, dtype=torch.int32, device=dev)
    mine[: blob.size] = torch.from_numpy(blob).to(dev)
    got = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(got, mine, group=group)
    recs = np.zeros((S, T, k, 8), np.int32)
    nrec = np.zeros((S, T), np.int32)
    navail = np.zeros((S, T), np.int64)
    allreqs = []
    for g, sz in zip(got, sizes):
        b = g.cpu().numpy()[: int(sz.item())]
        ns, off = int(b[0]), 1
        for _ in range(ns):
            idx = int(b[off])
            nrec[idx] = b[off + 1: off + 1 + T]
            navail[idx] = b[off + 1 + T: off + 1 + 3 * T].copy().view(np.int64)
            recs[idx] = b[off + 1 + 3 * T: off + per].reshape(T, k, 8)
            off += per
        allreqs.append(b[off:].reshape(-1, 19))
    _tick(timing, "allgather", t0)
    local = {srv.my_server_idx: srv for srv in servers}
    return settle(local, servers[0].num_app_ranks, servers[0].user_types, k, recs, nrec, navail,
                  np.concatenate(allreqs), timing)


# ------------------------------------------------------------------ steal group
class StealGroup:
    """The steal round of the shards this process holds, in the library
    (adlbq_steal_group_*): one device blob for every shard's export, an
    optional all-gather of the blobs over RCCL (device buffers end to end),
    one copy to pinned memory, the merge and the per-shard grants / deletions
    without a per-shard synchronisation."""

    def __init__(self, servers, k: int, rqcap: int = 4096):
        self.lib = _lib.load()
        self.servers = list(servers)
        arr = (ctypes.c_void_p * len(self.servers))(*[s.h.value for s in self.servers])
        g = ctypes.c_void_p()
        _lib.check(self.lib.adlbq_steal_group_create(ctypes.byref(g), arr, len(self.servers), int(k), int(rqcap)),
                   "adlbq_steal_group_create")
        self.g = g
        self.blob_ints = int(self.lib.adlbq_steal_group_blob_ints(g))
        self._dblob = None
        self._gathered = None
        self._hblob = None
        self._hall = None

    def round(self, group=None, timing=None):
        """One steal round.  Single process: the local blob is merged as it is;
        with a process group: the blobs are all-gathered first -- device
        tensors end to end over RCCL ("nccl"), or through pinned host memory
        over a host backend (gloo; adlbq_steal_group_export_host / _settle_host,
        the path a node's MPI server processes take).  Returns (decided,
        settled) over all shards."""
        import torch
        import torch.distributed as dist
        t0 = time.perf_counter()
        multi = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
        if multi and dist.get_backend(group) != "nccl":
            return self._round_host(group, timing, t0)
        if not multi:
            self.export_device(None)
            t0 = _tick(timing, "export", t0)
            out = self.settle_device(None, 1)
            _tick(timing, "merge_apply", t0)
            return out
        if self._dblob is None:
            dev = torch.device("cuda", torch.cuda.current_device())
            self._dblob = torch.empty(self.blob_ints, dtype=torch.int32, device=dev)
            self._gathered = torch.empty(dist.get_world_size(group) * self.blob_ints, dtype=torch.int32, device=dev)
        self.export_device(self._dblob.data_ptr())
        # the export runs on the shards' streams: the collective's stream waits for them
        for s in self.servers:
            s.sync()
        dist.all_gather_into_tensor(self._gathered, self._dblob, group=group)
        torch.cuda.current_stream().synchronize()
        t0 = _tick(timing, "export", t0)
        out = self.settle_device(self._gathered.data_ptr(), dist.get_world_size(group))
        _tick(timing, "merge_apply", t0)
        return out

    def export_device(self, d_blob):
        """The device half of a round's first step: every local shard's export
        into the device buffer d_blob (blob_ints int32; None: an internal one),
        enqueued on the shards' streams (adlbq_steal_group_export)."""
        _lib.check(self.lib.adlbq_steal_group_export(self.g, d_blob), "adlbq_steal_group_export")

    def settle_device(self, d_all, nproc: int):
        """The settle over the device buffer d_all = [nproc][blob_ints] as
        all_gather_into_tensor lays the processes' blobs out (None with nproc 1:
        the last export): adlbq_steal_group_settle.  Returns (decided, settled)."""
        nd, ns = ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.adlbq_steal_group_settle(self.g, d_all, int(nproc), ctypes.byref(nd), ctypes.byref(ns)),
                   "adlbq_steal_group_settle")
        return nd.value, ns.value

    def _round_host(self, group, timing, t0):
        import torch
        import torch.distributed as dist
        w = dist.get_world_size(group)
        if self._hblob is None:
            self._hblob = torch.empty(self.blob_ints, dtype=torch.int32).pin_memory()
            self._hall = torch.empty(w * self.blob_ints, dtype=torch.int32)
        _lib.check(self.lib.adlbq_steal_group_export_host(self.g, self._hblob.data_ptr()),
                   "adlbq_steal_group_export_host")
        parts = list(self._hall.view(w, self.blob_ints).unbind(0))
        dist.all_gather(parts, self._hblob, group=group)
        t0 = _tick(timing, "export", t0)
        nd, ns = ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.adlbq_steal_group_settle_host(self.g, self._hall.data_ptr(), w, ctypes.byref(nd),
                                                          ctypes.byref(ns)), "adlbq_steal_group_settle_host")
        _tick(timing, "merge_apply", t0)
        return nd.value, ns.value

    def responses(self) -> np.ndarray:
        c = ctypes.c_int()
        _lib.check(self.lib.adlbq_steal_group_responses(self.g, 0, None, ctypes.byref(c)), "responses")
        out = np.empty((c.value, 15), np.int32)
        if c.value:
            _lib.check(self.lib.adlbq_steal_group_responses(self.g, c.value, out.ctypes.data, ctypes.byref(c)),
                       "responses")
        return out

    def grants(self) -> np.ndarray:
        """(m, 3) {local shard j, rank, wqseqno} pinned by the last round"""
        c = ctypes.c_int()
        _lib.check(self.lib.adlbq_steal_group_grants(self.g, 0, None, ctypes.byref(c)), "grants")
        out = np.empty((c.value, 3), np.int32)
        if c.value:
            _lib.check(self.lib.adlbq_steal_group_grants(self.g, c.value, out.ctypes.data, ctypes.byref(c)), "grants")
        return out

    def unreserve_grants(self):
        _lib.check(self.lib.adlbq_steal_group_unreserve_grants(self.g), "adlbq_steal_group_unreserve_grants")

    def stat(self, name: str) -> int:
        return int(self.lib.adlbq_steal_group_stat(self.g, name.encode()))

    def check(self):
        a, b = ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.adlbq_steal_group_check(self.g, ctypes.byref(a), ctypes.byref(b)), "check")
        return a.value, b.value

    def close(self):
        if getattr(self, "g", None):
            self.lib.adlbq_steal_group_destroy(self.g)
            self.g = None
