"""ctypes binding of the ADLB server core (adlb_amd/csrc/adlb_core.h, libadlbsrv.so).

The core is the server's message handlers without MPI: each method takes one
inbound message (or a run of Reserves / Gets) and returns the replies the
server sends, as (dest world rank, tag, bytes) in sending order.  libadlb.so's
MPI loop drives the same handlers; tests drive them with event streams
recorded from the reference server (tests/test_gpu_server.py).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libadlbsrv.so")
HEADER = os.path.join(HERE, "csrc", "adlb_core.h")

P, c_int, c_double = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
EMIT = ctypes.CFUNCTYPE(None, ctypes.c_void_p, c_int, c_int, ctypes.c_void_p, c_int)

SIGNATURES = {
    "adlbsrv_create": (c_int, [P, c_int, P, c_int, c_int, c_int, c_double, c_int, EMIT, P]),
    "adlbsrv_destroy": (c_int, [P]),
    "adlbsrv_last_error": (ctypes.c_char_p, []),
    "adlbsrv_put_hdr": (c_int, [P, c_int, P, P]),
    "adlbsrv_put_payload": (c_int, [P, c_int, P, P, c_int]),
    "adlbsrv_put_stage": (c_int, [P, c_int, P, P, c_int]),
    "adlbsrv_put_flush": (c_int, [P]),
    "adlbsrv_put_staged": (c_int, [P]),
    "adlbsrv_put_common_hdr": (c_int, [P, c_int, c_int, P]),
    "adlbsrv_put_common_payload": (c_int, [P, c_int, P, c_int]),
    "adlbsrv_batch_done": (c_int, [P, c_int, c_int, c_int]),
    "adlbsrv_get_common": (c_int, [P, c_int, c_int]),
    "adlbsrv_did_put_at_remote": (c_int, [P, c_int, c_int, c_int]),
    "adlbsrv_reserve_batch": (c_int, [P, c_int, P, P]),
    "adlbsrv_get_batch": (c_int, [P, c_int, P, P]),
    "adlbsrv_info_num": (c_int, [P, c_int, c_int]),
    "adlbsrv_no_more_work": (c_int, [P]),
    "adlbsrv_exhausted": (c_int, [P]),
    "adlbsrv_qmstat": (c_int, [P, P, P, P]),
    "adlbsrv_my_row": (c_int, [P, P, P, P]),
    "adlbsrv_rfr": (c_int, [P, c_int, P]),
    "adlbsrv_rfr_resp": (c_int, [P, c_int, P]),
    "adlbsrv_unreserve": (c_int, [P, c_int, P]),
    "adlbsrv_push_tick": (c_int, [P]),
    "adlbsrv_push_query": (c_int, [P, c_int, P]),
    "adlbsrv_push_query_resp": (c_int, [P, c_int, P]),
    "adlbsrv_push_len": (c_int, [P, c_int]),
    "adlbsrv_push_hdr": (c_int, [P, c_int, P, P, c_int]),
    "adlbsrv_push_del": (c_int, [P, c_int, P]),
    "adlbsrv_moving_targeted": (c_int, [P, c_int, P]),
    "adlbsrv_num_parked": (c_int, [P]),
    "adlbsrv_activity": (ctypes.c_longlong, [P]),
    "adlbsrv_row_stamp": (ctypes.c_longlong, [P]),
    "adlbsrv_rfr_outstanding": (c_int, [P]),
    "adlbsrv_nmw": (c_int, [P]),
    "adlbsrv_info_get": (c_int, [P, c_int, P]),
    "adlbsrv_group_create": (c_int, [P, c_int, c_int]),
    "adlbsrv_group_blob_ints": (ctypes.c_longlong, [P]),
    "adlbsrv_group_export": (c_int, [P, P]),
    "adlbsrv_group_settle": (c_int, [P, P, c_int, P]),
    "adlbsrv_group_export_device": (c_int, [P, P]),
    "adlbsrv_group_settle_device": (c_int, [P, P, c_int, P]),
    "adlbsrv_group_stat": (ctypes.c_longlong, [P, c_int]),
    "adlbsrv_replay_many": (c_int, [P, c_int, c_int, P, P, P, P, P, P]),
    "adlbsrv_replay_prof": (None, [P]),
    "adlbsrv_replay_rounds": (c_int, [P, c_int, c_int, P, P, c_int, c_int, P, P, P, P, ctypes.c_longlong, P, P, P]),
    "adlbsrv_replay_rounds2": (c_int, [P, c_int, c_int, P, P, c_int, c_int, P, P, P, P, ctypes.c_longlong, P, P, P,
                                       c_int, P]),
    "adlbsrv_replay_error": (ctypes.c_char_p, []),
}

_lib = None


class CoreError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise CoreError(f"{LIB_PATH} is missing: build it with __graft_entry__.build()")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        _lib = lib
    return _lib


def _i32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.int32))


class Core:
    """One server rank's handlers.  Every call returns the list of replies."""

    def __init__(self, user_types, num_app_ranks: int, num_servers: int, my_world_rank: int,
                 max_malloc: float = 1e12, device: int = 0):
        lib = load()
        self._out: list[tuple[int, int, bytes]] = []

        def _emit(ctx, dest, tag, buf, n):
            self._out.append((dest, tag, ctypes.string_at(buf, n) if n > 0 else b""))

        self._cb = EMIT(_emit)   # keep the callback alive
        self._types = _i32(user_types)
        self.T = self._types.size
        self.S = num_servers
        h = ctypes.c_void_p()
        self._chk(lib.adlbsrv_create(ctypes.byref(h), self.T, self._types.ctypes.data, num_app_ranks, num_servers,
                                     my_world_rank, float(max_malloc), device, self._cb, None), "create")
        self._h = h

    def _chk(self, rc, what):
        if rc < 0:
            raise CoreError(f"adlbsrv_{what}: {load().adlbsrv_last_error().decode(errors='replace')}")
        return rc

    def _take(self):
        out, self._out = self._out, []
        return out

    def put(self, src: int, hdr12, payload: bytes):
        h = _i32(hdr12)
        need = c_int()
        self._chk(load().adlbsrv_put_hdr(self._h, src, h.ctypes.data, ctypes.byref(need)), "put_hdr")
        if need.value:
            b = ctypes.create_string_buffer(payload, len(payload))
            self._chk(load().adlbsrv_put_payload(self._h, src, h.ctypes.data, b, len(payload)), "put_payload")
        return self._take()

    def put_run(self, puts):
        """A run of FA_PUT_HDRs as libadlb.so's loop drains it: each header
        checked and acked in turn, the accepted payloads staged, then one
        engine batch (adlbsrv_put_stage / adlbsrv_put_flush).  puts: [(src,
        hdr12, payload)]."""
        lib = load()
        need = c_int()
        for src, hdr12, payload in puts:
            h = _i32(hdr12)
            self._chk(lib.adlbsrv_put_hdr(self._h, src, h.ctypes.data, ctypes.byref(need)), "put_hdr")
            if need.value:
                b = ctypes.create_string_buffer(payload, len(payload))
                self._chk(lib.adlbsrv_put_stage(self._h, src, h.ctypes.data, b, len(payload)), "put_stage")
        self._chk(lib.adlbsrv_put_flush(self._h), "put_flush")
        assert lib.adlbsrv_put_staged(self._h) == 0
        return self._take()

    def put_common(self, src: int, common_len: int, payload: bytes):
        need = c_int()
        self._chk(load().adlbsrv_put_common_hdr(self._h, src, common_len, ctypes.byref(need)), "put_common_hdr")
        if need.value:
            b = ctypes.create_string_buffer(payload, len(payload))
            self._chk(load().adlbsrv_put_common_payload(self._h, src, b, len(payload)), "put_common_payload")
        return self._take()

    def batch_done(self, src, cqseqno, refcnt):
        self._chk(load().adlbsrv_batch_done(self._h, src, cqseqno, refcnt), "batch_done")
        return self._take()

    def get_common(self, src, cqseqno):
        self._chk(load().adlbsrv_get_common(self._h, src, cqseqno), "get_common")
        return self._take()

    def did_put_at_remote(self, work_type, target, server_rank):
        self._chk(load().adlbsrv_did_put_at_remote(self._h, work_type, target, server_rank), "did_put_at_remote")
        return self._take()

    def reserve_batch(self, srcs, bufs17):
        s, b = _i32(srcs), _i32(bufs17).reshape(-1, 17)
        self._chk(load().adlbsrv_reserve_batch(self._h, s.size, s.ctypes.data, b.ctypes.data), "reserve_batch")
        return self._take()

    def get_batch(self, srcs, wqseqnos):
        s, w = _i32(srcs), _i32(wqseqnos)
        self._chk(load().adlbsrv_get_batch(self._h, s.size, s.ctypes.data, w.ctypes.data), "get_batch")
        return self._take()

    def info_num(self, src, work_type):
        self._chk(load().adlbsrv_info_num(self._h, src, work_type), "info_num")
        return self._take()

    def no_more_work(self):
        self._chk(load().adlbsrv_no_more_work(self._h), "no_more_work")
        return self._take()

    def exhausted(self):
        self._chk(load().adlbsrv_exhausted(self._h), "exhausted")
        return self._take()

    def qmstat(self, qlen, nbytes, hi):
        q, h = _i32(qlen), _i32(hi)
        nb = np.ascontiguousarray(np.asarray(nbytes, np.float64))
        self._chk(load().adlbsrv_qmstat(self._h, q.ctypes.data, nb.ctypes.data, h.ctypes.data), "qmstat")
        return self._take()

    def my_row(self):
        q, nb, hi = c_int(), c_double(), np.zeros(max(self.T, 1), np.int32)
        self._chk(load().adlbsrv_my_row(self._h, ctypes.byref(q), ctypes.byref(nb), hi.ctypes.data), "my_row")
        return q.value, nb.value, hi[: self.T]

    def rfr(self, src, buf28):
        b = _i32(buf28)
        self._chk(load().adlbsrv_rfr(self._h, src, b.ctypes.data), "rfr")
        return self._take()

    def rfr_resp(self, src, buf28):
        b = _i32(buf28)
        self._chk(load().adlbsrv_rfr_resp(self._h, src, b.ctypes.data), "rfr_resp")
        return self._take()

    def unreserve(self, src, buf12):
        b = _i32(buf12)
        self._chk(load().adlbsrv_unreserve(self._h, src, b.ctypes.data), "unreserve")
        return self._take()

    # -- memory-pressure push (adlb.c:509-556, 2109-2362) ------------------------------
    def push_tick(self):
        """The loop-top check; returns (sent, replies)."""
        sent = self._chk(load().adlbsrv_push_tick(self._h), "push_tick")
        return sent, self._take()

    def push_query(self, src, d12):
        d = np.ascontiguousarray(np.asarray(d12, np.float64))
        self._chk(load().adlbsrv_push_query(self._h, src, d.ctypes.data), "push_query")
        return self._take()

    def push_query_resp(self, src, d12):
        d = np.ascontiguousarray(np.asarray(d12, np.float64))
        self._chk(load().adlbsrv_push_query_resp(self._h, src, d.ctypes.data), "push_query_resp")
        return self._take()

    def push_len(self, wqseqno) -> int:
        return load().adlbsrv_push_len(self._h, int(wqseqno))

    def push_hdr(self, src, buf12, payload: bytes):
        b = _i32(buf12)
        p = ctypes.create_string_buffer(payload, max(len(payload), 1))
        self._chk(load().adlbsrv_push_hdr(self._h, src, b.ctypes.data, p, len(payload)), "push_hdr")
        return self._take()

    def push_del(self, src, buf12):
        b = _i32(buf12)
        self._chk(load().adlbsrv_push_del(self._h, src, b.ctypes.data), "push_del")
        return self._take()

    def moving_targeted(self, src, buf12):
        b = _i32(buf12)
        self._chk(load().adlbsrv_moving_targeted(self._h, src, b.ctypes.data), "moving_targeted")
        return self._take()

    def num_parked(self) -> int:
        return load().adlbsrv_num_parked(self._h)

    def info_get(self, key: int) -> float:
        v = c_double()
        self._chk(load().adlbsrv_info_get(self._h, key, ctypes.byref(v)), "info_get")
        return v.value

    def close(self):
        if getattr(self, "_h", None):
            load().adlbsrv_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
