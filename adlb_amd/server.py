"""Host-side mirror of one ADLB server's queue handlers over the C ABI.

Each method corresponds to a handler site of the reference server loop
(``src/adlb.c``) and to one entry point of ``include/adlbq.h``; the matching
itself runs in the HIP library (``adlb_amd/libadlbq.so``).  Arguments and
results keep the reference's meaning: world ranks, user work-type values,
TA_RESERVE_RESP int[12] records, NULL/-1 for "not found".
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

RESP_INTS = 12
PUT_INTS = 9
RESERVE_INTS = 18
LOWEST_PRIO = -999999999


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


class Server:
    """Queue state of one ADLB server rank on one MI355X (ADLBP_Init's per-server
    setup, adlb.c:295-320)."""

    def __init__(self, user_types, num_app_ranks: int, num_servers: int = 1, my_server_idx: int = 0,
                 max_units: int = 1 << 16, device: int = 0):
        self.lib = _lib.load()
        ut = np.ascontiguousarray(np.asarray(user_types, dtype=np.int32))
        self.user_types = ut
        self.T = int(ut.size)
        self.num_app_ranks = int(num_app_ranks)
        self.num_servers = int(num_servers)
        self.my_server_idx = int(my_server_idx)
        h = ctypes.c_void_p()
        _lib.check(self.lib.adlbq_create(ctypes.byref(h), self.T, _ptr(ut), self.num_app_ranks,
                                         self.num_servers, self.my_server_idx, int(max_units), int(device)),
                   "adlbq_create")
        self.h = h

    # -- lifecycle -------------------------------------------------------------
    def close(self):
        if getattr(self, "h", None):
            self.lib.adlbq_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    # -- FA_PUT_HDR (adlb.c:963-1046) -----------------------------------------
    def put_batch(self, units9) -> np.ndarray:
        """units9: (n, 9) {type, prio, answer_rank, target_rank, len, home_server,
        common_len, common_server, common_seqno} -> (n, 3) {wqseqno, matched_rank,
        matched_rqseqno}."""
        u = np.ascontiguousarray(np.asarray(units9, dtype=np.int32).reshape(-1, PUT_INTS))
        out = np.empty((u.shape[0], 3), dtype=np.int32)
        _lib.check(self.lib.adlbq_put_batch(self.h, u.shape[0], _ptr(u), _ptr(out)), "adlbq_put_batch")
        return out

    def put_batch_device(self, units9, d_out3: int) -> None:
        """adlbq_put_batch_device: results {wqseqno, matched_rank, matched_rqseqno}
        land in device memory at d_out3 (n x 3 int32), in stream order."""
        u = np.ascontiguousarray(np.asarray(units9, dtype=np.int32).reshape(-1, PUT_INTS))
        _lib.check(self.lib.adlbq_put_batch_device(self.h, u.shape[0], _ptr(u), int(d_out3)), "adlbq_put_batch_device")

    def put(self, work_type, prio, answer_rank=0, target_rank=-1, length=8, home_server=-1,
            common_len=0, common_server=-1, common_seqno=-1):
        return self.put_batch([[work_type, prio, answer_rank, target_rank, length, home_server,
                                common_len, common_server, common_seqno]])[0]

    # -- FA_RESERVE (adlb.c:1199-1317) ----------------------------------------
    def reserve_batch(self, reqs18) -> np.ndarray:
        """reqs18: (n, 18) {from_rank, hang, req_types[16]} -> (n, 12) TA_RESERVE_RESP
        (+ [10] rqseqno if parked, [11] RFR target server rank)."""
        r = np.ascontiguousarray(np.asarray(reqs18, dtype=np.int32).reshape(-1, RESERVE_INTS))
        out = np.empty((r.shape[0], RESP_INTS), dtype=np.int32)
        _lib.check(self.lib.adlbq_reserve_batch(self.h, r.shape[0], _ptr(r), _ptr(out)),
                   "adlbq_reserve_batch")
        return out

    def reserve(self, rank, req_types, hang=1):
        tv = list(req_types)[:16]
        tv += [-2] * (16 - len(tv))
        return self.reserve_batch([[rank, hang] + tv])[0]

    def reserve_batch_device(self, n: int, d_reqs: int, d_resp: int) -> None:
        """Device-pointer variant (HBM-resident requests/responses, stream ordered)."""
        _lib.check(self.lib.adlbq_reserve_batch_device(self.h, n, d_reqs, d_resp),
                   "adlbq_reserve_batch_device")

    # -- FA_GET_RESERVED / SS_UNRESERVE ---------------------------------------
    def get_reserved(self, rank, wqseqno):
        out = np.empty(5, dtype=np.int32)
        _lib.check(self.lib.adlbq_get_reserved(self.h, rank, wqseqno, _ptr(out)), "adlbq_get_reserved")
        return out

    def get_reserved_batch(self, pairs) -> np.ndarray:
        """FA_GET_RESERVED for (n, 2) {rank, wqseqno} pairs in arrival order -> (n, 5)."""
        p = np.ascontiguousarray(np.asarray(pairs, dtype=np.int32).reshape(-1, 2))
        out = np.empty((p.shape[0], 5), dtype=np.int32)
        _lib.check(self.lib.adlbq_get_reserved_batch(self.h, p.shape[0], _ptr(p), _ptr(out)),
                   "adlbq_get_reserved_batch")
        return out

    def get_reserved_batch_device(self, n: int, d_pairs2: int, d_out5: int) -> None:
        _lib.check(self.lib.adlbq_get_reserved_batch_device(self.h, n, d_pairs2, d_out5),
                   "adlbq_get_reserved_batch_device")

    def unreserve(self, rank, wqseqno, new_pin_rank=-1) -> int:
        f = ctypes.c_int()
        _lib.check(self.lib.adlbq_unreserve(self.h, rank, wqseqno, new_pin_rank, ctypes.byref(f)),
                   "adlbq_unreserve")
        return f.value

    def unreserve_batch_device(self, n: int, d_triples: int) -> None:
        _lib.check(self.lib.adlbq_unreserve_batch_device(self.h, n, d_triples),
                   "adlbq_unreserve_batch_device")

    def unreserve_resp_device(self, n: int, d_reqs18: int, d_resp12: int) -> None:
        """SS_UNRESERVE every unit the reserve batch (d_reqs18, d_resp12) matched."""
        _lib.check(self.lib.adlbq_unreserve_resp_device(self.h, n, d_reqs18, d_resp12),
                   "adlbq_unreserve_resp_device")

    # -- qmstat / donor selection ----------------------------------------------
    def qmstat_row(self):
        q = ctypes.c_int()
        hi = np.empty(max(self.T, 1), dtype=np.int32)
        _lib.check(self.lib.adlbq_qmstat_row(self.h, ctypes.byref(q), _ptr(hi)), "adlbq_qmstat_row")
        return q.value, hi[: self.T].copy()

    def set_qmstat_row(self, server_idx, qlen, nbytes_used, type_hi_prio):
        hi = np.ascontiguousarray(np.asarray(type_hi_prio, dtype=np.int32))
        _lib.check(self.lib.adlbq_set_qmstat_row(self.h, server_idx, qlen, float(nbytes_used), _ptr(hi)),
                   "adlbq_set_qmstat_row")

    def check_remote(self) -> np.ndarray:
        cap = 1 << 16
        out = np.empty((cap, 3), dtype=np.int32)
        k = ctypes.c_int()
        _lib.check(self.lib.adlbq_check_remote(self.h, cap, _ptr(out), ctypes.byref(k)), "adlbq_check_remote")
        return out[: k.value].copy()

    def rfr_done(self, from_server_rank, for_rank):
        _lib.check(self.lib.adlbq_rfr_done(self.h, from_server_rank, for_rank), "adlbq_rfr_done")

    def tq_add(self, app_rank, work_type, server_rank):
        _lib.check(self.lib.adlbq_tq_add(self.h, app_rank, work_type, server_rank), "adlbq_tq_add")

    def rq_delete(self, rqseqno) -> int:
        f = ctypes.c_int()
        _lib.check(self.lib.adlbq_rq_delete(self.h, rqseqno, ctypes.byref(f)), "adlbq_rq_delete")
        return f.value

    def push_select(self, threshold):
        c, s = ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.adlbq_push_select(self.h, float(threshold), ctypes.byref(c), ctypes.byref(s)),
                   "adlbq_push_select")
        return c.value, s.value

    # -- push protocol (adlb.c:2109-2362) -------------------------------------------
    def push_accept(self, unit9) -> int:
        """SS_PUSH_QUERY at the pushee: the unit held for this server; its wqseqno."""
        u = np.ascontiguousarray(np.asarray(unit9, dtype=np.int32).reshape(PUT_INTS))
        s = ctypes.c_int()
        _lib.check(self.lib.adlbq_push_accept(self.h, _ptr(u), ctypes.byref(s)), "adlbq_push_accept")
        return s.value

    def push_take(self, wqseqno) -> np.ndarray:
        """SS_PUSH_QUERY_RESP at the pusher: {ok, type, prio, len, answer, target, home, clen, csrv, cseq}."""
        out = np.zeros(10, dtype=np.int32)
        _lib.check(self.lib.adlbq_push_take(self.h, int(wqseqno), _ptr(out)), "adlbq_push_take")
        return out

    def push_commit(self, wqseqno) -> np.ndarray:
        """SS_PUSH_HDR at the pushee: {found, matched_rank, matched_rqseqno}."""
        out = np.zeros(3, dtype=np.int32)
        _lib.check(self.lib.adlbq_push_commit(self.h, int(wqseqno), _ptr(out)), "adlbq_push_commit")
        return out

    def push_discard(self, wqseqno) -> int:
        f = ctypes.c_int()
        _lib.check(self.lib.adlbq_push_discard(self.h, int(wqseqno), ctypes.byref(f)), "adlbq_push_discard")
        return f.value

    # -- steal round (adlb_amd/shards.py) ----------------------------
    def steal_export(self, k: int):
        """Per type, the k best available units (SS_RFR donor side for every request
        at once): (recs [T, k, 8] {prio, wqseqno, type, len, answer, common_len,
        common_server, common_seqno}, nrec [T], navail [T] int64)."""
        recs = np.empty((max(self.T, 1), int(k), 8), dtype=np.int32)
        nrec = np.empty(max(self.T, 1), dtype=np.int32)
        navail = np.empty(max(self.T, 1), dtype=np.int64)
        _lib.check(self.lib.adlbq_steal_export(self.h, int(k), _ptr(recs), _ptr(nrec), _ptr(navail)),
                   "adlbq_steal_export")
        return recs[: self.T], nrec[: self.T], navail[: self.T]

    def steal_begin(self, k: int) -> None:
        """Enqueue the export (top-k per type + live rq entries); steal_collect() waits."""
        _lib.check(self.lib.adlbq_steal_begin(self.h, int(k)), "adlbq_steal_begin")
        self._steal_k = int(k)

    def steal_collect(self):
        """-> (recs [T, k, 8], nrec [T], navail [T], rq (n, 18)) of the export in flight."""
        k = self._steal_k
        recs = np.empty((max(self.T, 1), k, 8), dtype=np.int32)
        nrec = np.empty(max(self.T, 1), dtype=np.int32)
        navail = np.empty(max(self.T, 1), dtype=np.int64)
        cap = getattr(self, "_rq_cap_hint", 1024)
        rq = np.empty((cap, 18), dtype=np.int32)
        c = ctypes.c_int()
        _lib.check(self.lib.adlbq_steal_collect(self.h, _ptr(recs), _ptr(nrec), _ptr(navail), cap, _ptr(rq),
                                                ctypes.byref(c)), "adlbq_steal_collect")
        if c.value > cap:   # only the first cap entries were copied: take the rest the slow way
            self._rq_cap_hint = 2 * c.value
            rq = self.rq_export()
        else:
            rq = rq[: c.value].copy()
        return recs[: self.T], nrec[: self.T], navail[: self.T], rq

    def steal_apply(self, pairs2, rqseqnos) -> None:
        """Enqueue this shard's side of a settled round: pin the granted (rank,
        wqseqno) pairs, drop the settled rq entries (no host synchronisation)."""
        p = np.ascontiguousarray(np.asarray(pairs2, dtype=np.int32).reshape(-1, 2))
        q = np.ascontiguousarray(np.asarray(rqseqnos, dtype=np.int32).ravel())
        _lib.check(self.lib.adlbq_steal_apply(self.h, p.shape[0], _ptr(p), q.size, _ptr(q)), "adlbq_steal_apply")

    def steal_check(self):
        """Synchronise; (grants whose unit was gone, rqseqnos no longer parked) since the last check."""
        a, b = ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.adlbq_steal_check(self.h, ctypes.byref(a), ctypes.byref(b)), "adlbq_steal_check")
        return a.value, b.value

    def rq_export(self) -> np.ndarray:
        """Live parked Reserves in rqseqno order: (n, 18) {rqseqno, world_rank, req_types[16]}."""
        cap = 1024
        while True:
            out = np.empty((cap, 18), dtype=np.int32)
            c = ctypes.c_int()
            _lib.check(self.lib.adlbq_rq_export(self.h, cap, _ptr(out), ctypes.byref(c)), "adlbq_rq_export")
            if c.value <= cap:
                return out[: c.value].copy()
            cap = c.value

    def grant_batch(self, pairs2) -> np.ndarray:
        """Pin (rank, wqseqno) pairs the merge granted (adlb.c:1820-1824) -> found[n]."""
        p = np.ascontiguousarray(np.asarray(pairs2, dtype=np.int32).reshape(-1, 2))
        found = np.empty(p.shape[0], dtype=np.int32)
        _lib.check(self.lib.adlbq_grant_batch(self.h, p.shape[0], _ptr(p), _ptr(found)), "adlbq_grant_batch")
        return found

    def rq_delete_batch(self, rqseqnos) -> np.ndarray:
        q = np.ascontiguousarray(np.asarray(rqseqnos, dtype=np.int32).ravel())
        found = np.empty(q.size, dtype=np.int32)
        _lib.check(self.lib.adlbq_rq_delete_batch(self.h, q.size, _ptr(q), _ptr(found)), "adlbq_rq_delete_batch")
        return found

    # -- info --------------------------------------------------------------------
    def info(self):
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.adlbq_info(self.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), "adlbq_info")
        return a.value, b.value, c.value

    def bytes(self):
        """(curr, hwm): the handle's share of curr_bytes_dmalloced / hwm_bytes_dmalloced."""
        c, h = ctypes.c_double(), ctypes.c_double()
        _lib.check(self.lib.adlbq_bytes(self.h, ctypes.byref(c), ctypes.byref(h)), "adlbq_bytes")
        return c.value, h.value

    def bytes_adjust(self, delta: float) -> None:
        _lib.check(self.lib.adlbq_bytes_adjust(self.h, float(delta)), "adlbq_bytes_adjust")

    def put_check(self, work_len: int, max_malloc: float):
        """FA_PUT_HDR's memory check: (rejected, hint_server_rank)."""
        r, hnt = ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.adlbq_put_check(self.h, int(work_len), float(max_malloc), ctypes.byref(r),
                                            ctypes.byref(hnt)), "adlbq_put_check")
        return r.value, hnt.value

    def info_type(self, work_type):
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.check(self.lib.adlbq_info_type(self.h, work_type, ctypes.byref(a), ctypes.byref(b),
                                            ctypes.byref(c)), "adlbq_info_type")
        return a.value, b.value, c.value

    # -- plumbing ------------------------------------------------------------------
    def set_stream(self, stream_ptr: int | None):
        _lib.check(self.lib.adlbq_set_stream(self.h, stream_ptr or None), "adlbq_set_stream")

    def sync(self):
        _lib.check(self.lib.adlbq_sync(self.h), "adlbq_sync")

    def profile(self, on=True):
        _lib.check(self.lib.adlbq_profile_enable(self.h, 1 if on else 0), "adlbq_profile_enable")

    def profile_only(self, stage: str | None):
        _lib.check(self.lib.adlbq_profile_only(self.h, stage.encode() if stage else None), "adlbq_profile_only")

    def profile_read(self, stage: str):
        ms, n = ctypes.c_double(), ctypes.c_longlong()
        _lib.check(self.lib.adlbq_profile_read(self.h, stage.encode(), ctypes.byref(ms), ctypes.byref(n)),
                   "adlbq_profile_read")
        return ms.value, n.value

    def stat(self, name: str) -> int:
        return int(self.lib.adlbq_stat(self.h, name.encode()))

    def last_scan_units(self) -> int:
        return int(self.lib.adlbq_last_scan_units(self.h))

    def set_param(self, name: str, value: int) -> None:
        """Tuning knobs of the engine (adlbq_set_param); results never depend on them."""
        _lib.check(self.lib.adlbq_set_param(self.h, name.encode(), int(value)), "adlbq_set_param")


class ReserveGroup:
    """adlbq_reserve_group_device over a fixed set of one process's server
    shards: every shard's Reserve batch as one launch per pipeline kernel
    (include/adlbq.h).  pack() builds a call's argument arrays once, so a
    loop over pre-staged batches does no per-call marshalling."""

    def __init__(self, servers):
        self.servers = list(servers)
        self.n = len(self.servers)
        self.lib = self.servers[0].lib
        self._hs = (ctypes.c_void_p * self.n)(*[s.h for s in self.servers])

    def pack(self, counts, d_reqs, d_resp):
        n = self.n
        if not (len(counts) == len(d_reqs) == len(d_resp) == n):
            raise ValueError("one count, request pointer and reply pointer per shard")
        return ((ctypes.c_void_p * n)(*d_reqs), (ctypes.c_void_p * n)(*d_resp), (ctypes.c_int * n)(*counts))

    def reserve_device(self, counts=None, d_reqs=None, d_resp=None, packed=None) -> None:
        rq, rs, ct = packed if packed is not None else self.pack(counts, d_reqs, d_resp)
        _lib.check(self.lib.adlbq_reserve_group_device(self._hs, self.n, rq, rs, ct), "adlbq_reserve_group_device")

    def unreserve_resp_device(self, counts=None, d_reqs=None, d_resp=None, packed=None) -> None:
        """adlbq_unreserve_resp_group_device: SS_UNRESERVE of every unit the shards' batches matched."""
        rq, rs, ct = packed if packed is not None else self.pack(counts, d_reqs, d_resp)
        _lib.check(self.lib.adlbq_unreserve_resp_group_device(self._hs, self.n, rq, rs, ct),
                   "adlbq_unreserve_resp_group_device")
