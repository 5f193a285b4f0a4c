"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV directory.

usage: python tools/step_timeline.py <rocprofv3 output dir>

A step ends at each k_unreserve_resp launch (the last kernel of a bench step);
the last five complete steps without a copy (the device-resident timed region,
not the host-buffer batches the bench runs after it) are averaged per kernel
position.  'span' is the
first kernel start to the last kernel end of a step, 'busy' the sum of the
kernel durations (the difference is the idle time between kernels).
"""
import csv
import glob
import sys


def main(d):
    f = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    # a step ends with its unreserve launch (the bench's step = reserve batch + unreserve)
    idx = [i + 1 for i, r in enumerate(rows) if "k_unreserve_resp" in r["Kernel_Name"]]
    steps = [rows[a:b] for a, b in zip(idx[:-1], idx[1:])]
    steps = [st for st in steps if not any("copyBuffer" in r["Kernel_Name"] for r in st)][-5:]
    agg = {}
    gaps = {}
    for st in steps:
        prev = None
        for n, r in enumerate(st):
            agg.setdefault((n, r["Kernel_Name"][:60]), []).append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
            gaps.setdefault(n, []).append(0.0 if prev is None else (int(r["Start_Timestamp"]) - prev) / 1000)
            prev = int(r["End_Timestamp"])
    for (n, name), v in sorted(agg.items()):
        g = gaps.get(n, [0.0])
        print(f"{n:2d} {name:60s} {sum(v) / len(v):8.2f} us  (gap before {sum(g) / len(g):5.2f}, max {max(v):7.2f})")
    spans = [(int(st[-1]["End_Timestamp"]) - int(st[0]["Start_Timestamp"])) / 1000 for st in steps]
    busy = [sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in st) / 1000 for st in steps]
    print(f"step span {sum(spans) / len(spans):.1f} us, busy {sum(busy) / len(busy):.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
