"""Build-container timing of the reference's src/xq.c (oracle/_ref/libxqref.so)
beside this repo's restatement (oracle/liboracle.so) on the same queues:
seconds per Reserve and ns per node visit (2 x units per Reserve: the
pre-targeted scan, xq.c:219-247, then wq_find_hi_prio, xq.c:190-217).
  python tools/oracle_ref_timing.py > profiles/r02_oracle_ref_vs_port.json
"""
import json
import os
import platform
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle.baseline import sample  # noqa: E402

out = {"host": platform.processor() or platform.machine(), "cpus": os.cpu_count(), "runs": []}
out["note"] = ("the reference build keeps its queue under adlb.c's own allocation cap (max_malloc = 500 MB until "
               "ADLB_Server sets it, adlb.c:218): 10M units (~1.3 GB with payloads) abort it, so 10M is timed "
               "on the restatement only")
for n_units in (100_000, 1_000_000, 3_000_000, 10_000_000):
    for kind in (("ref", "own") if n_units * 150 < 4.5e8 else ("own",)):
        done, el, held = sample((kind, n_units, 4, 65536, 1000, False, 0, 1, 6.0 if n_units > 100_000 else 3.0))
        per = el / max(done, 1)
        out["runs"].append({"kind": kind, "units": held, "reserves": done, "s_per_reserve": per,
                            "ns_per_node": per / (2.0 * held) * 1e9, "reserves_per_s": done / el})
        print(out["runs"][-1], file=sys.stderr, flush=True)
print(json.dumps(out, indent=1))
