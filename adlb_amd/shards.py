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

`reduce_step_timing` is the bench's max-over-ranks / sum-over-ranks reduction.
"""
from __future__ import annotations

import numpy as np


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
