"""Wall time of relinked applications next to the reference build (GPU box).

The reference's examples/nq.c and examples/tsp.c run unchanged (a) against the
reference library (oracle/_ref/nq_plain, tsp_plain: examples + src/adlb.c +
src/xq.c compiled where they lie, no recorder) and (b) relinked against
adlb_amd/libadlb.so (oracle/_ref/nq_amd, tsp_amd), under the same mpirun on the
same host, with the answer checked on every run.  libadlb.so variants: Put
batching on / off (ADLB_PUT_BATCH) and the steal group off / on
(ADLB_STEAL_GROUP).

The deep-queue case (tests/apps/adlb_deep.c) is matching-dominated: every unit
is queued before the first Reserve, and `app_time` is its Reserve/Get phase.

nq and tsp both end by exhaustion, which the reference detects after a 5 s
quiet qmstat ring (adlb.c:490, 754-785) and libadlb.so after two 0.5 s polls,
so the wall times are dominated by that detection delay; nq also prints its
own compute time ("time ..."), reported per run as `app_time`.

  python tools/app_timing.py [--reps 3] > profiles/r04_app_timing.json
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")
GOLD = os.path.join(ROOT, "tests", "golden")
MPIRUN = "/opt/conda/bin/mpirun"


def run(binary, np_, args, stdin=None, env_extra=None, timeout=600):
    env = dict(os.environ, ADLB_DEVICE="0", **(env_extra or {}))
    fin = open(stdin) if stdin else None
    t0 = time.perf_counter()
    r = subprocess.run([MPIRUN, "-np", str(np_), binary, *args], stdin=fin, env=env, capture_output=True, text=True,
                       timeout=timeout)
    el = time.perf_counter() - t0
    if fin:
        fin.close()
    if r.returncode != 0:
        raise RuntimeError(f"{binary} rc={r.returncode}: {r.stdout[-1500:]} {r.stderr[-1500:]}")
    return el, r.stdout


def deep_ok(n):
    def ok(out):
        ln = [x for x in out.splitlines() if x.startswith("adlb_deep:")]
        if not ln:
            return False
        v = ln[0].split()
        return v[2] == v[6] == str(n) and v[4] == v[7]
    return ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", default="", help="run only the cases whose name starts with this")
    args = ap.parse_args()
    with open(os.path.join(GOLD, "tsp_expected.json")) as f:
        tsp_exp = json.load(f)
    cases = [
        ("nq -n 9, 2 servers, 4 apps", "nq", 6, ["-n", "9", "-q", "-nservers", "2"], None,
         lambda out: "found 352 solutions" in out),
        ("nq -n 11, 2 servers, 6 apps", "nq", 8, ["-n", "11", "-q", "-nservers", "2"], None,
         lambda out: "found 2680 solutions" in out),
        ("tsp 11 cities, 2 servers, 3 apps", "tsp", 5, ["-nservers", "2"], os.path.join(GOLD, "tsp_m11.txt"),
         lambda out: f"bdist {tsp_exp['tsp_m11.txt']['reference_bdist']}" in out),
        # matching-dominated: every unit queued before any Reserve (tests/apps/adlb_deep.c); the
        # reference scans its xq list per Reserve, the engine matches the waiting Reserves together
        ("deep queue 40000 units, 1 server, 4 apps", "deep", 5, ["-n", "40000"], None, deep_ok(40000)),
        ("deep queue 20000 units, 1 server, 8 apps", "deep", 9, ["-n", "20000"], None, deep_ok(20000)),
    ]
    cases = [c for c in cases if c[0].startswith(args.only)]
    variants = [("reference", "_plain", None),
                ("libadlb.so", "_amd", {"ADLB_PUT_BATCH": "1", "ADLB_STEAL_GROUP": "0"}),
                ("libadlb.so, one engine call per Put", "_amd", {"ADLB_PUT_BATCH": "0", "ADLB_STEAL_GROUP": "0"}),
                ("libadlb.so, steal group", "_amd", {"ADLB_PUT_BATCH": "1", "ADLB_STEAL_GROUP": "1"})]
    res = {"host_cpus": len(os.sched_getaffinity(0)), "reps": args.reps, "cases": []}
    for name, app, np_, a, stdin, ok in cases:
        row = {"case": name, "np": np_, "args": a, "seconds": {}}
        for vname, suffix, env in variants:
            b = os.path.join(REF, app + suffix)
            if app == "deep" and suffix == "_amd":
                b = os.path.join(ROOT, "tests", "apps", "adlb_deep")
            if not os.path.exists(b):
                row["seconds"][vname] = None
                continue
            ts, at = [], []
            for _ in range(args.reps):
                el, out = run(b, np_, a, stdin, env)
                if not ok(out):
                    raise RuntimeError(f"{vname} {name}: wrong answer\n{out[-1500:]}")
                ts.append(round(el, 3))
                m = [ln for ln in out.splitlines() if "solutions, time" in ln or ln.startswith("adlb_deep:")]
                if m:
                    at.append(float(m[0].split()[-1]))
            row["seconds"][vname] = {"min": min(ts), "all": ts}
            if at:
                row["seconds"][vname]["app_time"] = at
            print(f"{name:40s} {vname:40s} {min(ts):8.3f} s", file=sys.stderr, flush=True)
        if app == "tsp":
            row["note"] = ("ends by exhaustion: the reference waits for a 5 s quiet qmstat ring, libadlb.so for two "
                           "0.5 s polls")
        res["cases"].append(row)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
