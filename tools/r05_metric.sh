#!/bin/bash
# Round 5: parity subset, then the metric leg under adlbq_set_param variants and a
# rocprofv3 kernel trace of the default (medians per kernel).
#   bash tools/r05_metric.sh "<pytest -k expr or empty>" "chain_seq=0" "chain_seq=1" ...
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r05m
mkdir -p $O
K="$1"; shift
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -k "$K" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
i=0
for v in "$@"; do
  i=$((i+1))
  P=""
  for kv in $(echo $v | tr ',' ' '); do P="$P --param $kv"; done
  timeout -k 10 300 python3 bench.py --no-cpu --no-host-path --no-config3 --no-config4 --no-config5 --no-wide --no-pmc $EXTRA $P > $O/v$i.json 2> $O/v$i.err || { echo "variant $v failed"; tail -5 $O/v$i.err; exit 1; }
  python3 - "$O/v$i.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {s: v["ms"] for s, v in d["kernels_ms"].items()}
print(f"{sys.argv[2]:30s} ms/step {d['ms_per_step']:.4f} parity {d['parity']} kernels {k}")
if d.get("chain_last_batch"): print("   chain", d.get("chain_last_batch"))
PY
done
if [ -n "$PROF" ]; then
  rm -rf $O/p
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/p -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-pmc --no-host-path --no-config3 --no-config4 --no-config5 --no-wide > $O/prof.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
  f=$(find $O/p -name "*kernel_trace.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
r = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for x in r:
    d[x['Kernel_Name'][:48] + ' g' + x['Grid_Size_X']].append(int(x['End_Timestamp']) - int(x['Start_Timestamp']))
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    if len(v) >= 10: print(f"{k:64s} n={len(v):4d} median={sorted(v)[len(v) // 2] / 1000:.1f}us")
PY
fi
