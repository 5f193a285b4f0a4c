"""Replay an event trace (format of oracle/replay.h) through the C ABI.

Consecutive Puts become one ``adlbq_put_batch``, consecutive Reserves one
``adlbq_reserve_batch`` and consecutive Gets one ``adlbq_get_reserved_batch``
-- the batch entry points guarantee the same results as
processing the events one at a time, so the output stream must equal the
oracle's byte for byte.
"""
from __future__ import annotations

import numpy as np

from .server import Server
from .synth import (OP_BYTES, OP_CHECKREM, OP_GET, OP_HWM, OP_INFO, OP_INFOTYPE, OP_PUSHACCEPT, OP_PUSHCOMMIT,
                    OP_PUSHDEL, OP_PUSHSEL, OP_PUSHTAKE, OP_PUT, OP_PUTCHECK, OP_QMROW, OP_RESERVE, OP_RFRDONE,
                    OP_RQDEL, OP_SETROW, OP_TQADD, OP_UNRESERVE)


def nargs(op: int, T: int) -> int:
    return {OP_PUT: 9, OP_RESERVE: 18, OP_GET: 2, OP_UNRESERVE: 3, OP_QMROW: 0, OP_SETROW: 3 + T,
            OP_CHECKREM: 0, OP_RFRDONE: 2, OP_TQADD: 3, OP_PUSHSEL: 1, OP_INFO: 0, OP_RQDEL: 1,
            OP_INFOTYPE: 1, OP_BYTES: 0, OP_PUTCHECK: 2, OP_HWM: 0, OP_PUSHACCEPT: 9, OP_PUSHTAKE: 1,
            OP_PUSHCOMMIT: 1, OP_PUSHDEL: 1}[op]


def _runs(tr: np.ndarray, T: int):
    """Yield (op, args (k, nargs) array) for maximal runs of identical opcodes
    (PUT/RESERVE) and single events otherwise."""
    i, n = 0, tr.size
    while i < n:
        op = int(tr[i])
        w = 1 + nargs(op, T)
        if op in (OP_PUT, OP_RESERVE, OP_GET):
            j = i
            # stride through the run while the opcode repeats
            while j < n and int(tr[j]) == op:
                j += w
            block = tr[i:j].reshape(-1, w)
            yield op, block[:, 1:]
            i = j
        else:
            yield op, tr[i + 1:i + w].reshape(1, -1)
            i += w


def event_prefix(tr: np.ndarray, T: int, n_ints: int) -> int:
    """Length of the longest prefix of whole events with at most n_ints ints
    (at least the first event): a cut that never splits an event."""
    i = 0
    while i < tr.size:
        w = 1 + nargs(int(tr[i]), T)
        if i + w > n_ints and i > 0:
            break
        i += w
    return min(i, tr.size)


def replay(srv: Server, trace) -> np.ndarray:
    tr = np.ascontiguousarray(np.asarray(trace, dtype=np.int32))
    T = srv.T
    out: list[np.ndarray] = []

    def emit(vals):
        v = np.asarray(vals, dtype=np.int32).ravel()
        out.append(np.concatenate([np.asarray([v.size], np.int32), v]))

    for op, a in _runs(tr, T):
        if op == OP_PUT:
            r = srv.put_batch(a)
            blk = np.empty((r.shape[0], 4), np.int32)
            blk[:, 0] = 3
            blk[:, 1:] = r
            out.append(blk.ravel())
        elif op == OP_RESERVE:
            r = srv.reserve_batch(a)
            blk = np.empty((r.shape[0], 13), np.int32)
            blk[:, 0] = 12
            blk[:, 1:] = r
            out.append(blk.ravel())
        elif op == OP_GET:
            r = srv.get_reserved_batch(a)
            blk = np.empty((r.shape[0], 6), np.int32)
            blk[:, 0] = 5
            blk[:, 1:] = r
            out.append(blk.ravel())
        else:
            x = [int(v) for v in a[0]]
            if op == OP_UNRESERVE:
                emit([srv.unreserve(x[0], x[1], x[2])])
            elif op == OP_QMROW:
                q, hi = srv.qmstat_row()
                emit([q, *hi.tolist()])
            elif op == OP_SETROW:
                srv.set_qmstat_row(x[0], x[1], x[2], x[3:3 + T])
                emit([])
            elif op == OP_CHECKREM:
                r = srv.check_remote()
                emit([r.shape[0], *r.ravel().tolist()])
            elif op == OP_RFRDONE:
                srv.rfr_done(x[0], x[1])
                emit([])
            elif op == OP_TQADD:
                srv.tq_add(x[0], x[1], x[2])
                r = srv.check_remote()  # adlb.c:1179
                emit([r.shape[0], *r.ravel().tolist()])
            elif op == OP_PUSHSEL:
                emit(list(srv.push_select(x[0])))
            elif op == OP_INFO:
                emit(list(srv.info()))
            elif op == OP_RQDEL:
                emit([srv.rq_delete(x[0])])
            elif op == OP_INFOTYPE:
                emit(list(srv.info_type(x[0])))
            elif op == OP_BYTES:
                emit([int(srv.bytes()[0])])
            elif op == OP_HWM:
                emit([int(srv.bytes()[1])])
            elif op == OP_PUTCHECK:
                emit(list(srv.put_check(x[0], x[1])))
            elif op == OP_PUSHACCEPT:
                emit([srv.push_accept(x)])
            elif op == OP_PUSHTAKE:
                emit(srv.push_take(x[0]).tolist())
            elif op == OP_PUSHCOMMIT:
                emit(srv.push_commit(x[0]).tolist())
            elif op == OP_PUSHDEL:
                emit([srv.push_discard(x[0])])
            else:
                raise ValueError(f"unknown opcode {op}")
    return np.concatenate(out) if out else np.zeros(0, np.int32)


def replay_many(servers, traces, cap_factor: int = 8):
    """The traces of several shards replayed at once by the native driver
    (adlb_amd/csrc/adlb_replay.cpp, one host thread per shard, each handle on
    its own stream): the same calls and output stream as replay() per shard.
    Returns (outputs, ABI calls per shard)."""
    import ctypes

    from . import core
    lib = core.load()
    n = len(servers)
    trs = [np.ascontiguousarray(np.asarray(t, dtype=np.int32)) for t in traces]
    outs = [np.empty(cap_factor * t.size + (1 << 20), np.int32) for t in trs]
    PA = ctypes.c_void_p * n
    LA = ctypes.c_longlong * n
    hs = PA(*[s.h.value if hasattr(s.h, "value") else s.h for s in servers])
    tp = PA(*[t.ctypes.data for t in trs])
    lens = LA(*[t.size for t in trs])
    op = PA(*[o.ctypes.data for o in outs])
    caps = LA(*[o.size for o in outs])
    nout, ncall = LA(), LA()
    T = servers[0].T
    rc = lib.adlbsrv_replay_many(hs, n, T, tp, lens, op, caps, nout, ncall)
    if rc:  # -2: an output buffer was too small (the servers have moved on: no retry)
        raise RuntimeError(f"adlbsrv_replay_many: {lib.adlbsrv_replay_error().decode(errors='replace')}")
    return [o[: nout[j]].copy() for j, o in enumerate(outs)], [ncall[j] for j in range(n)]


def replay_rounds(servers, traces, k: int, rqcap: int, steal_cap: int = 1 << 22, closed: bool = False,
                  stats: dict | None = None):
    """Config 5 at its SURVEY shape (adlb_replay.cpp, adlbsrv_replay_rounds): the
    shards' traces with steal rounds (event 23 in every trace), device-side
    batches between the rounds from one host thread per shard, one steal-group
    round (export depth k, rqcap parked Reserves per shard) at each marker.
    closed: a Get is issued only once the reply it depends on has landed, with
    the wqseqno from that reply (adlbsrv_replay_rounds2); stats then receives
    {get_calls_waited, wait_s, wqseqno_mismatch}.
    Returns (outputs per shard, steals (n, 15), seconds, calls per shard)."""
    import ctypes

    from . import core
    lib = core.load()
    n = len(servers)
    trs = [np.ascontiguousarray(np.asarray(t, dtype=np.int32)) for t in traces]
    outs = [np.empty(2 * t.size + (1 << 20), np.int32) for t in trs]
    steals = np.empty((steal_cap, 15), np.int32)
    PA = ctypes.c_void_p * n
    LA = ctypes.c_longlong * n
    hs = PA(*[s.h.value if hasattr(s.h, "value") else s.h for s in servers])
    tp = PA(*[t.ctypes.data for t in trs])
    lens = LA(*[t.size for t in trs])
    op = PA(*[o.ctypes.data for o in outs])
    caps = LA(*[o.size for o in outs])
    nout, ncall = LA(), LA()
    nst = ctypes.c_longlong()
    sec = ctypes.c_double()
    cl = (ctypes.c_double * 3)()
    rc = lib.adlbsrv_replay_rounds2(hs, n, servers[0].T, tp, lens, k, rqcap, op, caps, nout, steals.ctypes.data,
                                    steal_cap, ctypes.byref(nst), ctypes.byref(sec), ncall, 1 if closed else 0, cl)
    if stats is not None:
        stats.update(get_calls_waited=int(cl[0]), wait_s=round(cl[1], 4), wqseqno_mismatch=int(cl[2]))
    if rc:
        raise RuntimeError(f"adlbsrv_replay_rounds: {lib.adlbsrv_replay_error().decode(errors='replace')}")
    return ([o[: nout[j]].copy() for j, o in enumerate(outs)], steals[: nst.value].copy(), sec.value,
            [ncall[j] for j in range(n)])


def last_rounds_prof() -> dict:
    """Host seconds of the last replay_rounds, summed over the shards' threads
    (adlb_replay.cpp adlbsrv_replay_prof): per call kind, the round barrier
    (waiting + the round), the rounds alone, and the wall time."""
    import ctypes

    from . import core
    v = (ctypes.c_double * 8)()
    core.load().adlbsrv_replay_prof(v)
    return dict(zip(("put", "reserve", "get", "qmrow", "setrow", "barrier", "rounds", "wall"),
                    [round(x, 4) for x in v]))


def server_process(trace_path: str, out_path: str, user_types, num_app_ranks: int, num_servers: int, idx: int,
                   device: int, barrier, q) -> None:
    """One ADLB server as its own process (the reference runs one per MPI rank):
    loads its recorded stream, warms a throwaway handle up on a prefix, waits at
    the barrier with the other servers, replays the whole stream through the C
    ABI (native driver, adlb_replay.cpp) and reports (idx, t_start, t_end,
    calls); the outputs go to out_path.  Used by bench.py's config-5 leg."""
    import time
    try:
        tr = np.load(trace_path)
        with Server(user_types, num_app_ranks, num_servers, idx, max_units=1 << 16, device=device) as tmp:
            replay_many([tmp], [tr[: event_prefix(tr, len(user_types), 20000)]])
        with Server(user_types, num_app_ranks, num_servers, idx, max_units=1 << 16, device=device) as srv:
            barrier.wait(timeout=300)
            t0 = time.time()
            got, calls = replay_many([srv], [tr])
            t1 = time.time()
        np.save(out_path, got[0])
        q.put((idx, t0, t1, int(calls[0]), ""))
    except Exception as e:  # reported to the parent, which fails the leg
        try:
            barrier.abort()
        except Exception:
            pass
        q.put((idx, 0.0, 0.0, 0, f"{type(e).__name__}: {e}"))
