"""CPU checks of the ADLB server library (no GPU calls): libadlb.so exports the
whole public API the reference's libadlb.a does, the core
binding matches its header, and the recorded config-1 fixtures are
self-consistent."""
import os
import re
import subprocess

import numpy as np
import pytest

from nq_fixture import Fixture, normalise

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBADLB = os.path.join(ROOT, "adlb_amd", "libadlb.so")
HEADER = os.path.join(ROOT, "include", "adlb", "adlb.h")
GOLD = os.path.join(ROOT, "tests", "golden")


def _exports(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {ln.split()[-1] for ln in out.splitlines() if " T " in ln}


def test_libadlb_exports_public_api():
    if not os.path.exists(LIBADLB):
        pytest.skip("libadlb.so not built")
    exp = _exports(LIBADLB)
    declared = set(re.findall(r"^int\s+(ADLBP?_\w+)\s*\(", open(HEADER).read(), re.M))
    # the symbols the reference's examples and adlb_prof.c reach besides the header
    extra = {"adlbp_dbgprintf", "adlbp_Reserve", "adlbp_Get_reserved_timed", "adlbp_Probe", "adlb_Probe",
             "dmalloc", "dfree", "pmalloc"}
    missing = sorted((declared | extra) - exp)
    assert not missing, missing


# the Fortran bindings of reference src/adlbf.c:6-103 (lower-case + '_')
FORTRAN = ["adlb_init_", "adlb_server_", "adlb_debug_server_", "adlb_put_", "adlb_reserve_", "adlb_ireserve_",
           "adlb_get_reserved_", "adlb_get_reserved_timed_", "adlb_begin_batch_put_", "adlb_end_batch_put_",
           "adlb_begin_batch_put_2_", "adlb_end_batch_put_2_", "adlb_set_no_more_work_",
           "adlb_set_problem_done_", "adlb_info_get_", "adlb_info_num_work_units_", "adlb_finalize_",
           "adlb_abort_"]


def test_libadlb_exports_fortran_bindings():
    if not os.path.exists(LIBADLB):
        pytest.skip("libadlb.so not built")
    missing = sorted(set(FORTRAN) - _exports(LIBADLB))
    assert not missing, missing


def test_core_binding_covers_header():
    from adlb_amd import core
    txt = open(core.HEADER).read()
    declared = set(re.findall(r"\b(adlbsrv_[a-z_0-9]+)\s*\(", txt)) - {"adlbsrv_emit_fn"}
    assert declared == set(core.SIGNATURES)
    if os.path.exists(core.LIB_PATH):
        assert declared <= _exports(core.LIB_PATH)


FIXTURES = sorted(f for f in os.listdir(GOLD) if f.startswith(("nq_", "mix_")))


@pytest.mark.parametrize("name", FIXTURES)
def test_nq_fixture_consistent(name):
    fx = Fixture(os.path.join(GOLD, name))
    kinds = [e[0] for e in fx.events]
    exp = fx.expected()
    # every Put is acked twice (header, done), every Get answered with an ack and its payload
    puts, gets, res = kinds.count("put"), kinds.count("get"), kinds.count("reserve")
    acks = [x for x in exp if x[2] == 1020]
    assert len([a for a in acks if a[0] == "put"]) == 2 * puts
    assert len([x for x in exp if x[2] == 1010]) == gets
    # every Reserve is answered exactly once (immediately, by a Put, by exhaustion)
    assert len([x for x in exp if x[2] == 1008]) == res
    # a unit (server, wqseqno) is handed out once, by its own server or through a steal
    handed = [(normalise(*x)[2][6], normalise(*x)[2][5]) for x in exp if x[2] == 1008 and normalise(*x)[2][0] == 1]
    assert len(handed) == len(set(handed))
    if fx.S == 1:
        assert len(handed) == gets
    assert kinds.count("exhausted") == 1
    t = fx.types.tolist()
    # nq's types, adlb_mix's four, or adlb_mix -ntypes 100 (the four, then declared-only 1004 ...)
    assert t in ([1000, 2000, 3000], [11, 22, 33, 44]) or (t[:4] == [11, 22, 33, 44] and
                                                            t[4:] == [1000 + k for k in range(4, len(t))])


def test_mix_fixtures_cover_the_steal_paths():
    fx = [Fixture(os.path.join(GOLD, f)) for f in FIXTURES if f.startswith("mix_")]
    kinds = {e[0] for f in fx for e in f.events}
    # (SS_UNRESERVE needs a Put to win a race against an SS_RFR_RESP: recorded only sometimes)
    assert {"rfr", "rfr_resp", "common_hdr", "batch_done", "get_common", "info", "qmstat"} <= kinds
    fails = [e for f in fx for e in f.events if e[0] == "rfr_resp" and int(np.frombuffer(e[2][:4], np.int32)[0]) != 1]
    assert fails, "no failed SS_RFR_RESP recorded"
    many = [f for f in fx if len(f.types) > 64]
    assert many and any(e[0] == "rfr_resp" for f in many for e in f.events), "no >64-type steal recorded"
