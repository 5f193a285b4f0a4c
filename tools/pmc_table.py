"""Per-kernel table of the metric leg: rocprofv3 average duration, the bench's
HIP-event stage time and PMC HBM bytes per launch, against VERDICT r05's budgets.

usage: python tools/pmc_table.py <bench json line file> <rocprofv3 kernel_stats.csv> [bench json of the
       driver's shape for the ms/step line]
"""
import csv
import json
import sys

BUDGET = {"k_prep_hist": "<= 11 us", "k_thresholds": "-", "k_select_wave": "-", "k_rank": "in the chain's launch",
          "k_chain0": "<= 20 us", "k_rank_chain0": "<= 20 us (k_chain0's)",
          "k_finalize": "<= 6 us, <= 2x 56 B x R", "k_unreserve_resp": "-"}
STAGE = {"k_prep_hist": "hist", "k_thresholds": "thresholds", "k_select_wave": "select", "k_rank": "rank",
         "k_chain0": "chain", "k_rank_chain0": "chain", "k_finalize": "finalize"}


def last_json(path):
    with open(path) as f:
        return json.loads([ln for ln in f.read().splitlines() if ln.startswith("{")][-1])


def main(bench_path, stats_path, driver_path=None):
    b = last_json(bench_path)
    km = b.get("kernels_ms", {})
    rows = {}
    for r in csv.DictReader(open(stats_path)):
        name = r["Name"]
        base = name.split("(")[0].replace("void ", "").split("<")[0].strip()
        if base in BUDGET:
            rows[base] = float(r["AverageNs"]) / 1000
    R = b["config"]["reserves_per_step"]
    print("# Round-6 per-kernel table (metric leg, 10M units x 65,536 Reserves, T = 4): rocprofv3 average duration,")
    print("# the bench's HIP-event stage time and PMC HBM bytes per launch (two rocprofv3 --pmc passes:")
    print("# FETCH_SIZE doubled + WRITE_SIZE), against VERDICT r05's budgets")
    print(f"{'kernel':22s} {'rocprof us':>10s} {'event us':>9s} {'PMC MB':>8s} {'GB/s':>7s}  budget")
    for k in ("k_prep_hist", "k_thresholds", "k_select_wave", "k_rank", "k_chain0", "k_rank_chain0", "k_finalize",
              "k_unreserve_resp"):
        if k not in rows:
            continue
        st = km.get(STAGE.get(k, ""), {})
        ev = st.get("ms")
        tr = st.get("traffic")
        gbs = (tr / (rows[k] * 1e-6) / 1e9) if tr else None
        print(f"{k:22s} {rows[k]:10.1f} {ev * 1e3 if ev else float('nan'):9.1f} "
              f"{tr / 1e6 if tr else float('nan'):8.1f} {gbs if gbs else float('nan'):7.0f}  {BUDGET[k]}")
    fin = km.get("finalize", {}).get("traffic")
    if fin:
        print(f"\nfinalize traffic / (56 B x R = {56 * R / 1e6:.2f} MB): {fin / (56 * R):.1f}x")
    d = last_json(driver_path) if driver_path else b
    print(f"metric ({d['steps']} steps, {d['warmup']} warm-up): {d['ms_per_step']:.4f} ms/step, "
          f"{d['value']:.3e} assignments/s (VERDICT r05 target <= 0.080 ms/step at --steps 20)")


if __name__ == "__main__":
    main(*sys.argv[1:])
