"""Every bench step's span from a rocprofv3 --kernel-trace CSV directory.

usage: python tools/steps_trace.py <rocprofv3 output dir> [first] [count]

A step ends with its k_unreserve_resp launch.  For each step: the idle gap
before its first kernel (since the previous step's last kernel ended), its span
(first kernel start to last kernel end) and the kernels' busy time.  [first,
first + count) selects the steps summed at the end (the bench's timed region is
steps warmup + profiled .. + steps).
"""
import csv
import glob
import sys


def main(d, first=None, count=None):
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [0] + [i + 1 for i, r in enumerate(rows) if "k_unreserve_resp" in r["Kernel_Name"]]
    steps = [rows[a:b] for a, b in zip(idx[:-1], idx[1:])]
    prev_end = None
    tot = []
    for n, st in enumerate(steps):
        s0, s1 = int(st[0]["Start_Timestamp"]), int(st[-1]["End_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in st) / 1000
        gap = (s0 - prev_end) / 1000 if prev_end is not None else 0.0
        prev_end = s1
        sel = first is not None and first <= n < first + count
        if sel:
            tot.append((gap, (s1 - s0) / 1000, busy))
        print(f"{n:3d} kernels {len(st):2d} gap {gap:9.1f} us  span {(s1 - s0) / 1000:7.1f} us  busy {busy:6.1f} us"
              + ("  *" if sel else ""))
    if tot:
        g, s, b = (sum(x[i] for x in tot) for i in range(3))
        print(f"selected {len(tot)} steps: gaps {g:.1f} us, spans {s:.1f} us, busy {b:.1f} us, "
              f"(gaps after the first + spans) / steps = {(g - tot[0][0] + s) / len(tot):.2f} us")


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], int(a[1]) if len(a) > 1 else None, int(a[2]) if len(a) > 2 else None)
