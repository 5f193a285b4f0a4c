#!/bin/bash
# Round 4: kernel stats of the config-4 leg (extra bench.py arguments pass through)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r04c4prof
mkdir -p $O
python -c "import torch" > /dev/null 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --config4-only --no-cpu --no-pmc "$@" > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
r = list(csv.DictReader(open(sys.argv[1])))
for x in sorted(r, key=lambda x: -float(x['TotalDurationNs']))[:28]:
    print(x['Name'][:70], x['Calls'], x['AverageNs'])
PY
