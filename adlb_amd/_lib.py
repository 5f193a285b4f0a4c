"""ctypes binding of the C ABI in include/adlbq.h (adlb_amd/libadlbq.so).

The library is the product: HIP kernels for gfx950 behind a C ABI.  There is
no CPU fallback -- if the shared object is missing or fails to load, every
entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ADLBQ_LIB") or os.path.join(HERE, "libadlbq.so")  # override: experiments only
HEADER = os.path.join(os.path.dirname(HERE), "include", "adlbq.h")

c_int, c_ll, c_void_p, c_double, c_char_p = (ctypes.c_int, ctypes.c_longlong, ctypes.c_void_p,
                                            ctypes.c_double, ctypes.c_char_p)
P = ctypes.c_void_p

SIGNATURES = {
    "adlbq_create": (c_int, [P, c_int, P, c_int, c_int, c_int, c_ll, c_int]),
    "adlbq_destroy": (c_int, [P]),
    "adlbq_put_batch": (c_int, [P, c_int, P, P]),
    "adlbq_put_batch_device": (c_int, [P, c_int, P, P]),
    "adlbq_reserve_batch": (c_int, [P, c_int, P, P]),
    "adlbq_reserve_batch_device": (c_int, [P, c_int, P, P]),
    "adlbq_reserve_group_device": (c_int, [P, c_int, P, P, P]),
    "adlbq_get_reserved": (c_int, [P, c_int, c_int, P]),
    "adlbq_get_reserved_batch": (c_int, [P, c_int, P, P]),
    "adlbq_get_reserved_batch_device": (c_int, [P, c_int, P, P]),
    "adlbq_unreserve": (c_int, [P, c_int, c_int, c_int, P]),
    "adlbq_unreserve_batch_device": (c_int, [P, c_int, P]),
    "adlbq_unreserve_resp_device": (c_int, [P, c_int, P, P]),
    "adlbq_unreserve_resp_group_device": (c_int, [P, c_int, P, P, P]),
    "adlbq_qmstat_row": (c_int, [P, P, P]),
    "adlbq_set_qmstat_row": (c_int, [P, c_int, c_int, c_double, P]),
    "adlbq_check_remote": (c_int, [P, c_int, P, P]),
    "adlbq_rfr_done": (c_int, [P, c_int, c_int]),
    "adlbq_rfr_done_batch": (c_int, [P, c_int, P]),
    "adlbq_tq_add": (c_int, [P, c_int, c_int, c_int]),
    "adlbq_rq_delete": (c_int, [P, c_int, P]),
    "adlbq_tq_dec": (c_int, [P, c_int, c_int, c_int]),
    "adlbq_rfr_failed": (c_int, [P, c_int, c_int, P]),
    "adlbq_rfr_retry": (c_int, [P, c_int, P, P]),
    "adlbq_unit_target": (c_int, [P, c_int, P]),
    "adlbq_steal_export": (c_int, [P, c_int, P, P, P]),
    "adlbq_rq_export": (c_int, [P, c_int, P, P]),
    "adlbq_steal_begin": (c_int, [P, c_int]),
    "adlbq_steal_collect": (c_int, [P, P, P, P, c_int, P, P]),
    "adlbq_steal_apply": (c_int, [P, c_int, P, c_int, P]),
    "adlbq_steal_check": (c_int, [P, P, P]),
    "adlbq_push_accept": (c_int, [P, P, P]),
    "adlbq_set_qmstat_nbytes": (c_int, [P, c_int, c_double]),
    "adlbq_push_take": (c_int, [P, c_int, P]),
    "adlbq_push_commit": (c_int, [P, c_int, P]),
    "adlbq_push_discard": (c_int, [P, c_int, P]),
    "adlbq_steal_merge": (c_int, [c_int, c_int, P, c_int, P, P, P, c_int, P, P, P]),
    "adlbq_grant_batch": (c_int, [P, c_int, P, P]),
    "adlbq_steal_group_create": (c_int, [P, P, c_int, c_int, c_int]),
    "adlbq_steal_group_blob_ints": (c_ll, [P]),
    "adlbq_steal_group_export": (c_int, [P, P]),
    "adlbq_steal_group_settle": (c_int, [P, P, c_int, P, P]),
    "adlbq_steal_group_export_host": (c_int, [P, P]),
    "adlbq_steal_group_settle_host": (c_int, [P, P, c_int, P, P]),
    "adlbq_steal_group_responses": (c_int, [P, c_int, P, P]),
    "adlbq_steal_group_grants": (c_int, [P, c_int, P, P]),
    "adlbq_steal_group_check": (c_int, [P, P, P]),
    "adlbq_steal_group_unreserve_grants": (c_int, [P]),
    "adlbq_steal_group_stat": (c_ll, [P, c_char_p]),
    "adlbq_steal_group_destroy": (c_int, [P]),
    "adlbq_rq_delete_batch": (c_int, [P, c_int, P, P]),
    "adlbq_push_select": (c_int, [P, c_double, P, P]),
    "adlbq_info": (c_int, [P, P, P, P]),
    "adlbq_bytes": (c_int, [P, P, P]),
    "adlbq_bytes_adjust": (c_int, [P, c_double]),
    "adlbq_put_check": (c_int, [P, c_int, c_double, P, P]),
    "adlbq_info_type": (c_int, [P, c_int, P, P, P]),
    "adlbq_set_stream": (c_int, [P, P]),
    "adlbq_get_stream": (c_void_p, [P]),
    "adlbq_sync": (c_int, [P]),
    "adlbq_profile_enable": (c_int, [P, c_int]),
    "adlbq_profile_read": (c_int, [P, c_char_p, P, P]),
    "adlbq_profile_only": (c_int, [P, c_char_p]),
    "adlbq_last_scan_units": (c_ll, [P]),
    "adlbq_stat": (c_ll, [P, c_char_p]),
    "adlbq_set_param": (c_int, [P, c_char_p, c_ll]),
    "adlbq_last_error": (c_char_p, []),
    "adlbq_version": (c_char_p, []),
}

_lib = None


class AdlbqError(RuntimeError):
    pass


def header_symbols() -> list[str]:
    """Every function the public header declares."""
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"\b(adlbq_[a-z_0-9]+)\s*\(", txt)))


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise AdlbqError(f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                         "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().adlbq_last_error().decode(errors="replace")
        raise AdlbqError(f"{what} failed rc={rc}: {msg}")
