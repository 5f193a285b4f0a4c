"""TEST INFRASTRUCTURE ONLY -- the parity oracle.

Python handle onto the event-replay oracle (oracle/replay.c):

* ``Oracle("own")`` loads ``oracle/liboracle.so`` -- this repo's clean-room CPU
  restatement of the reference queue layer (``src/xq.c``) and of the server
  handlers in ``src/adlb.c``.  It is the checker used by ``tests/``,
  ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg, and it is
  the timed CPU baseline ("port").
* ``Oracle("ref")`` loads ``oracle/_ref/libxqref.so`` -- the same replay layer
  linked against the reference's own ``/root/reference/src/xq.c``.  It exists only
  in the build container and is used to generate/pin ``tests/golden``.

Nothing in ``adlb_amd/`` may import this package: the product path is the HIP
library and must fail loudly if it is missing.
"""
from __future__ import annotations

import ctypes
import os
import shutil
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LOWEST = -999999999
LIBS = {
    "own": os.path.join(HERE, "liboracle.so"),
    "ref": os.path.join(HERE, "_ref", "libxqref.so"),
}

OP_PUT, OP_RESERVE, OP_GET, OP_UNRESERVE, OP_QMROW, OP_SETROW = 1, 2, 3, 4, 5, 6
OP_CHECKREM, OP_RFRDONE, OP_TQADD, OP_PUSHSEL, OP_INFO, OP_RQDEL, OP_INFOTYPE = 7, 8, 9, 10, 11, 12, 13
OP_RFR, OP_RQLIST, OP_BYTES, OP_PUTCHECK, OP_HWM = 14, 15, 16, 17, 18
OP_PUSHACCEPT, OP_PUSHTAKE, OP_PUSHCOMMIT, OP_PUSHDEL = 19, 20, 21, 22
OP_ROUND = 23  # a steal round of the server group (gen_config5): outstanding RFR records cleared


def build(ref: bool = False) -> None:
    """Compile the oracle (and, when /root/reference exists, the reference build)."""
    subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)
    if ref and os.path.isdir("/root/reference/src"):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def available(kind: str = "own") -> bool:
    return os.path.exists(LIBS[kind])


class Oracle:
    """One ADLB server's queue state replayed on the CPU (single instance per
    process for the "ref" kind, since the reference keeps its queues in globals)."""

    def __init__(self, kind: str = "own", private: bool = False):
        """private=True loads a copy of the library, so that several servers
        (shards) can live in one process -- the replay state is global."""
        path = LIBS[kind]
        if not os.path.exists(path):
            if kind == "own":
                build()
            else:
                raise FileNotFoundError(f"{path} missing (make -C oracle ref)")
        self.kind = kind
        if private:
            tmp = tempfile.mkdtemp(prefix="oracle_")
            dst = os.path.join(tmp, os.path.basename(path))
            shutil.copy(path, dst)
            self.lib = ctypes.CDLL(dst, mode=ctypes.RTLD_LOCAL)
            shutil.rmtree(tmp, ignore_errors=True)   # the mapping stays valid
        else:
            self.lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        self.lib.orc_init.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                                      ctypes.c_int, ctypes.c_int]
        self.lib.orc_replay.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p,
                                        ctypes.c_long]
        self.lib.orc_replay.restype = ctypes.c_long

    def init(self, user_types, num_app_ranks: int, num_servers: int = 1, my_server_idx: int = 0):
        ut = np.ascontiguousarray(np.asarray(user_types, dtype=np.int32))
        self.ntypes = len(ut)
        self._ut = ut
        rc = self.lib.orc_init(len(ut), ut.ctypes.data, num_app_ranks, num_servers, my_server_idx)
        assert rc == 0

    def replay(self, trace) -> np.ndarray:
        tr = np.ascontiguousarray(np.asarray(trace, dtype=np.int32))
        cap = output_bound(tr, self.ntypes)
        out = np.empty(cap, dtype=np.int32)
        n = self.lib.orc_replay(tr.ctypes.data, tr.size, out.ctypes.data, cap)
        if n < 0:
            raise ValueError(f"oracle: malformed trace or output overflow (rc={n})")
        return out[:n].copy()

    def _one(self, op: int, *args, cap: int = 4096) -> np.ndarray:
        tr = np.asarray([op, *args], dtype=np.int32)
        out = np.empty(cap, dtype=np.int32)
        n = self.lib.orc_replay(tr.ctypes.data, tr.size, out.ctypes.data, cap)
        if n < 0:
            raise ValueError(f"oracle: event {op} failed (rc={n})")
        return out[1:1 + out[0]].copy()

    def qmrow(self):
        r = self._one(OP_QMROW)
        return int(r[0]), r[1:1 + self.ntypes]

    def rq_list(self) -> np.ndarray:
        """(n, 18) {rqseqno, rank, types[16]} in FIFO order."""
        nrq = int(self._one(OP_INFO)[2])
        r = self._one(OP_RQLIST, cap=64 + 18 * nrq)
        return r[1:].reshape(-1, 18)

    def rfr(self, rqseqno: int, for_rank: int, types16) -> np.ndarray:
        return self._one(OP_RFR, rqseqno, for_rank, *[int(x) for x in types16])

    def rqdel(self, rqseqno: int) -> int:
        return int(self._one(OP_RQDEL, rqseqno)[0])


def _find_cand_serial(me: int, types16, rows, user_types) -> int:
    """find_cand_rank_with_worktype (adlb.c:3487-3534) walked over the request's
    types in order (adlb.c:1280-1308) on a fresh table, no RFR outstanding and
    no tq entries.  Returns a shard index or -1."""
    for v in types16:
        v = int(v)
        if v < -1:
            break
        best, hi = -1, LOWEST
        for j, (qlen, row) in enumerate(rows):
            if j == me or qlen <= 0:
                continue
            if v < 0:
                for x in row:
                    if x > hi:
                        hi, best = int(x), j
            elif v in user_types:
                x = row[user_types.index(v)]
                if x > hi:
                    hi, best = int(x), j
        if best >= 0:
            return best
    return -1


def serial_steal_round(orcs, num_app_ranks: int) -> np.ndarray:
    """The steal round adlbq_steal_merge replaces, one RFR exchange at a time:
    the parked Reserves of shard 0, 1, ... in rqseqno order; each picks its
    donor on the current qmstat rows of every shard (update_local_state,
    adlb.c:3581-3593), the donor runs SS_RFR (adlb.c:1802-1866) and the
    requester SS_RFR_RESP (adlb.c:1868-1933: TA_RESERVE_RESP with the donor's
    world rank, rq_delete) before the next Reserve starts.
    Returns (n, 15) {shard, rqseqno, rank, TA_RESERVE_RESP[12]} per steal."""
    user_types = [int(x) for x in orcs[0]._ut]
    out = []
    for i, o in enumerate(orcs):
        for e in o.rq_list():
            rqseqno, rank, types = int(e[0]), int(e[1]), e[2:]
            rows = [x.qmrow() for x in orcs]
            d = _find_cand_serial(i, types, rows, user_types)
            if d < 0:
                continue
            r = orcs[d].rfr(rqseqno, rank, types)
            assert r[0] == 1, "a donor chosen on a fresh table must have a unit"
            assert o.rqdel(rqseqno) == 1
            out.append([i, rqseqno, rank, 1, r[3], r[4], r[5], r[6], r[7], num_app_ranks + d, r[9], r[10], r[11],
                        -1, -1])
    return np.asarray(out, dtype=np.int32).reshape(-1, 15)


def event_nargs(op: int, ntypes: int) -> int:
    return {OP_PUT: 9, OP_RESERVE: 18, OP_GET: 2, OP_UNRESERVE: 3, OP_QMROW: 0,
            OP_SETROW: 3 + ntypes, OP_CHECKREM: 0, OP_RFRDONE: 2, OP_TQADD: 3,
            OP_PUSHSEL: 1, OP_INFO: 0, OP_RQDEL: 1, OP_INFOTYPE: 1, OP_RFR: 18, OP_RQLIST: 0,
            OP_BYTES: 0, OP_PUTCHECK: 2, OP_HWM: 0, OP_PUSHACCEPT: 9, OP_PUSHTAKE: 1, OP_PUSHCOMMIT: 1,
            OP_PUSHDEL: 1, OP_ROUND: 0}[op]


def output_bound(tr: np.ndarray, ntypes: int) -> int:
    """Upper bound on replay output ints (the replay mutates state, so the buffer
    must be big enough the first time)."""
    for op, w in ((OP_PUT, 10), (OP_RESERVE, 19)):   # fast path: a pure run of one event kind
        if tr.size and tr.size % w == 0 and (tr[::w] == op).all():
            return 1024 + (tr.size // w) * (2 + max(12, ntypes + 1))
    ip, n_res, n_chk, n_ev = 0, 0, 0, 0
    trl = tr.tolist()
    while ip < len(trl):
        op = trl[ip]
        ip += 1 + event_nargs(op, ntypes)
        n_ev += 1
        n_res += op == OP_RESERVE
        n_chk += op in (OP_CHECKREM, OP_TQADD)
    return 1024 + n_ev * (2 + max(12, ntypes + 1)) + n_chk * (1 + 3 * n_res)


def gen_config5(n_shards: int = 8, n_ranks: int = 4096, n_events: int = 10_000_000, round_every: int = 10_000,
                k: int = 64, q0: int = 512, seed: int = 5, seed_units: int = 256) -> dict:
    """The config-5 stream at SURVEY §8(d)'s shape (oracle/gen_c5.c): per shard
    its event trace (a steal round = ORC_OP_ROUND at the same place in every
    shard's trace) and the oracle's outputs; the steals of every round
    {shard, rqseqno, rank, TA_RESERVE_RESP[12]} in serial order, and how many
    each round made; the generator's wall time (the oracle's CPU work)."""
    path = os.path.join(HERE, "libgen5.so")
    if not os.path.exists(path) or not os.path.exists(LIBS["own"]):
        subprocess.run(["make", "-s", "-C", HERE, "liboracle.so", "libgen5.so"], check=True)
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    lib.c5_new.restype = ctypes.c_void_p
    lib.c5_new.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           ctypes.c_ulonglong]
    lib.c5_error.restype = ctypes.c_char_p
    lib.c5_error.argtypes = [ctypes.c_void_p]
    lib.c5_run.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_long, ctypes.c_int]
    for f in ("c5_events", "c5_rounds", "c5_stopped"):
        getattr(lib, f).restype = ctypes.c_long
        getattr(lib, f).argtypes = [ctypes.c_void_p]
    lib.c5_seconds.restype = ctypes.c_double
    lib.c5_seconds.argtypes = [ctypes.c_void_p]
    pp = ctypes.POINTER(ctypes.POINTER(ctypes.c_int))
    for f in ("c5_trace", "c5_out", "c5_xtrace"):
        getattr(lib, f).restype = ctypes.c_long
        getattr(lib, f).argtypes = [ctypes.c_void_p, ctypes.c_int, pp]
    for f in ("c5_steals", "c5_round_nsteal"):
        getattr(lib, f).restype = ctypes.c_long
        getattr(lib, f).argtypes = [ctypes.c_void_p, pp]
    lib.c5_free.argtypes = [ctypes.c_void_p]
    g = lib.c5_new(LIBS["own"].encode(), n_shards, n_ranks, k, q0, seed)
    try:
        if lib.c5_run(g, n_events, round_every, seed_units) != 0:
            raise RuntimeError("gen_c5: " + lib.c5_error(g).decode())

        def arr(f, *a, cols=1):
            p = ctypes.POINTER(ctypes.c_int)()
            n = f(g, *a, ctypes.byref(p))
            return np.ctypeslib.as_array(p, shape=(n * cols,)).copy().reshape(-1, cols) if n else \
                np.zeros((0, cols), np.int32)

        return {"traces": [arr(lib.c5_trace, s).ravel() for s in range(n_shards)],
                "outputs": [arr(lib.c5_out, s).ravel() for s in range(n_shards)],
                # each shard's trace with its part of every steal round inlined (ORC_OP_RFR as donor,
                # ORC_OP_RQDEL as requester): one server process's whole work, replayed alone
                "xtraces": [arr(lib.c5_xtrace, s).ravel() for s in range(n_shards)],
                "steals": arr(lib.c5_steals, cols=15), "round_nsteal": arr(lib.c5_round_nsteal).ravel(),
                "events": lib.c5_events(g), "rounds": lib.c5_rounds(g), "stopped": lib.c5_stopped(g),
                "seconds": lib.c5_seconds(g), "n_shards": n_shards, "n_ranks": n_ranks, "k": k,
                "user_types": [1, 2]}
    finally:
        lib.c5_free(g)
