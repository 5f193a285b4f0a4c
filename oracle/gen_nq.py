"""TEST INFRASTRUCTURE ONLY -- config-1 fixtures from the reference itself.

Builds the reference's examples/nq.c with its own src/adlb.c + src/xq.c and
the PMPI recorder oracle/mpilog.c (`make -C oracle nqref`, output in the
gitignored oracle/_ref/), runs it under MPICH's mpirun exactly as SURVEY
§8(d) config 1 names it, and turns each server rank's message log into a
fixture under tests/golden/:

  nq_np4_n8.npz        mpirun -np 4 nq -n 8 -q                (1 server, 92 solutions)
  nq_np6_n9_s2_r4.npz  mpirun -np 6 nq -n 9 -q -nservers 2    (server rank 4 of 2, 352)
  nq_np6_n9_s2_r5.npz  ... server rank 5
  mix_np6_s2_r{4,5}.npz, mix_np7_s3_r{4,5,6}.npz   tests/apps/adlb_mix.c on the reference
                       library: steals, targeted work, a common-prefix batch
  mix_np6_s2_t100_r{4,5}.npz   the same with 100 declared work types (-ntypes 100): the
                       engine's >64-type path and SS_RFR steals

Fixture = the server's inbound events in the order its loop handled them and
every reply it sent, attributed to the event that caused it:
  meta        int64 {num_types, num_app_ranks, num_servers, my_world_rank, max_malloc}
  types       int32 [T]
  ev_kind/ev_src/ev_off/ev_len + ev_blob   inbound events (kinds: KINDS below)
  ex_ev/ex_dest/ex_tag/ex_off/ex_len + ex_blob   replies (event index, dest, tag, bytes)
Only the replies a handler decides are kept (TA_RESERVE_RESP, TA_ACK_AND_RC,
payloads, SS_RFR*, SS_UNRESERVE); the ring / timer traffic of the reference
(qmstat forwarding, end and exhaustion rings, debug timing) is not.  A
time-triggered exhaustion answer (adlb.c:757-772) becomes an `exhausted`
event of its own.

Run in the build container (needs /root/reference and /opt/conda's MPICH):
  python oracle/gen_nq.py [case ...]     (no case: all of them)
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
OUT = os.path.join(ROOT, "tests", "golden")

# inbound kinds of the fixture
KINDS = {"put": 1, "reserve": 2, "get": 3, "info": 4, "nmw": 5, "ss_nmw": 6, "qmstat": 7, "rfr": 8,
         "rfr_resp": 9, "unreserve": 10, "common_hdr": 11, "batch_done": 12, "get_common": 13,
         "did_put_at_remote": 14, "exhausted": 15}
# reference tags (src/adlb.c:44-83)
T_PUT_HDR, T_PUT_MSG, T_COMMON_HDR, T_COMMON_MSG, T_BATCH_DONE, T_DID_PUT = 1001, 1002, 1003, 1004, 1005, 1006
T_RESERVE, T_RESERVE_RESP, T_GET, T_GET_RESP, T_NMW = 1007, 1008, 1009, 1010, 1011
T_SS_NMW, T_QMSTAT, T_RFR, T_RFR_RESP, T_ACK, T_UNRESERVE = 1014, 1015, 1018, 1019, 1020, 1028
T_DONE_EXH, T_INFO, T_GET_COMMON, T_GET_COMMON_RESP = 1036, 1037, 1038, 1039
KEEP_OUT = {T_RESERVE_RESP, T_GET_RESP, T_ACK, T_RFR, T_RFR_RESP, T_UNRESERVE, T_GET_COMMON_RESP}
DONE_BY_EXHAUSTION = -999999998
NQ_TYPES = [1000, 2000, 3000]   # nq.c:44-46, 152
NQ_MAX_MALLOC = 25000000        # ADLB_Server(25000000, 0.0), nq.c:189


def parse_log(path):
    b = open(path, "rb").read()
    i, out = 0, []
    while i < len(b):
        h = np.frombuffer(b[i:i + 20], np.int32)
        i += 20
        n = int(h[4])
        out.append((int(h[0]), int(h[1]), int(h[2]), int(h[3]), b[i:i + n]))
        i += (n + 3) & ~3
    return out


def events_of(recs):
    """(events [(kind, src, bytes)], replies [(event index, dest, tag, bytes)])"""
    ev, ex = [], []
    for d, peer, tag, comm, data in recs:
        if d == 0:
            if tag == T_PUT_HDR:
                ev.append(["put", peer, data])
            elif tag == T_PUT_MSG:
                assert ev and ev[-1][0] == "put" and ev[-1][1] == peer, "payload without its header"
                ev[-1][2] = ev[-1][2] + data
            elif tag == T_COMMON_HDR:
                ev.append(["common_hdr", peer, data])
            elif tag == T_COMMON_MSG:
                assert ev and ev[-1][0] == "common_hdr" and ev[-1][1] == peer
                ev[-1][2] = ev[-1][2] + data
            elif tag in (T_RESERVE, T_GET, T_INFO, T_NMW, T_SS_NMW, T_QMSTAT, T_RFR, T_RFR_RESP, T_UNRESERVE,
                         T_BATCH_DONE, T_GET_COMMON, T_DID_PUT, T_DONE_EXH):
                kind = {T_RESERVE: "reserve", T_GET: "get", T_INFO: "info", T_NMW: "nmw", T_SS_NMW: "ss_nmw",
                        T_QMSTAT: "qmstat", T_RFR: "rfr", T_RFR_RESP: "rfr_resp", T_UNRESERVE: "unreserve",
                        T_BATCH_DONE: "batch_done", T_GET_COMMON: "get_common", T_DID_PUT: "did_put_at_remote",
                        T_DONE_EXH: "exhausted"}[tag]
                ev.append([kind, peer, data])
        elif tag in KEEP_OUT:
            if tag == T_RESERVE_RESP and np.frombuffer(data[:4], np.int32)[0] == DONE_BY_EXHAUSTION \
                    and (not ev or ev[-1][0] != "exhausted"):
                ev.append(["exhausted", -1, b""])   # the master's timer fired (adlb.c:754-772)
            assert ev, "a reply before any inbound message"
            ex.append((len(ev) - 1, peer, tag, data))
    return ev, ex


def write_fixture(path, ev, ex, A, S, me, types=NQ_TYPES, max_malloc=NQ_MAX_MALLOC):
    def pack(chunks):
        off = np.zeros(len(chunks), np.int64)
        ln = np.zeros(len(chunks), np.int64)
        pos = 0
        for i, c in enumerate(chunks):
            off[i], ln[i] = pos, len(c)
            pos += len(c)
        return off, ln, np.frombuffer(b"".join(chunks), np.uint8) if chunks else np.zeros(0, np.uint8)
    eo, el, eb = pack([e[2] for e in ev])
    xo, xl, xb = pack([x[3] for x in ex])
    np.savez_compressed(
        path, meta=np.array([len(types), A, S, me, max_malloc], np.int64),
        types=np.array(types, np.int32),
        ev_kind=np.array([KINDS[e[0]] for e in ev], np.int8), ev_src=np.array([e[1] for e in ev], np.int32),
        ev_off=eo, ev_len=el, ev_blob=eb,
        ex_ev=np.array([x[0] for x in ex], np.int32), ex_dest=np.array([x[1] for x in ex], np.int32),
        ex_tag=np.array([x[2] for x in ex], np.int32), ex_off=xo, ex_len=xl, ex_blob=xb)


def run_case(np_, args, servers, name, exe="nq", types=NQ_TYPES, max_malloc=NQ_MAX_MALLOC):
    subprocess.run(["make", "-s", "-C", HERE, "nqref" if exe == "nq" else f"_ref/{exe}"], check=True)
    with tempfile.TemporaryDirectory() as d:
        env = dict(os.environ, ADLB_MSGLOG_DIR=d)
        r = subprocess.run(["/opt/conda/bin/mpirun", "-np", str(np_), os.path.join(HERE, "_ref", exe), *args],
                           env=env, capture_output=True, text=True, timeout=300)
        found = [ln for ln in r.stdout.splitlines() if ln.startswith(("found", "adlb_mix"))]
        print(name, found)
        A = np_ - len(servers)
        for s in servers:
            ev, ex = events_of(parse_log(os.path.join(d, f"rank{s}.bin")))
            suffix = f"_r{s}" if len(servers) > 1 else ""
            path = os.path.join(OUT, f"{name}{suffix}.npz")
            write_fixture(path, ev, ex, A, len(servers), s, types, max_malloc)
            print(f"  {path}: {len(ev)} events, {len(ex)} replies")
        return found


MIX_TYPES = [11, 22, 33, 44]


def mix_types(k):
    """tests/apps/adlb_mix.c's declared types for -ntypes k"""
    return MIX_TYPES + [1000 + i for i in range(4, k)]


CASES = {
    "nq_np4_n8": lambda: run_case(4, ["-n", "8", "-q"], [3], "nq_np4_n8"),
    "nq_np6_n9_s2": lambda: run_case(6, ["-n", "9", "-q", "-nservers", "2"], [4, 5], "nq_np6_n9_s2"),
    # tests/apps/adlb_mix.c: steals (SS_RFR / SS_RFR_RESP / SS_UNRESERVE), targeted units,
    # a common-prefix batch, Ireserve and info queries (types 11, 22, 33, 44; hi 1e8)
    "mix_np6_s2": lambda: run_case(6, ["-nservers", "2", "-n", "200"], [4, 5], "mix_np6_s2", "mix", MIX_TYPES,
                                   100000000),
    "mix_np7_s3": lambda: run_case(7, ["-nservers", "3", "-n", "150"], [4, 5, 6], "mix_np7_s3", "mix", MIX_TYPES,
                                   100000000),
    # 100 declared types (more than the 64-bit type masks hold)
    "mix_np6_s2_t100": lambda: run_case(6, ["-nservers", "2", "-n", "120", "-ntypes", "100"], [4, 5],
                                        "mix_np6_s2_t100", "mix", mix_types(100), 100000000),
}


def main():
    if not os.path.isdir("/root/reference/src"):
        sys.exit("needs the reference sources (build container only)")
    for name in sys.argv[1:] or list(CASES):
        CASES[name]()


if __name__ == "__main__":
    main()
