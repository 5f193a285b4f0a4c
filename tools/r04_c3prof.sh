#!/bin/bash
# Round 4: rocprofv3 kernel stats of the config-3 leg (extra bench.py arguments pass through)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04c3p
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c3 -- python3 $R/bench.py --config3-only --no-pmc --no-cpu "$@" > $O/c3_bench.json 2> $O/c3.err || { echo c3 prof failed; tail -5 $O/c3.err; exit 1; }
cd $R
python3 - $O <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:22]:
    print(f'{r["Name"][:70]:70s} {r["Calls"]:>6s} {float(r["AverageNs"])/1e3:9.2f} us')
PY
