#!/bin/bash
# Round 4: metric leg with the request preparation and pass 1 as two launches (split_prep)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r04mdiag
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/p -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-pmc --no-host-path --no-config3 --no-config4 --no-config5 --no-wide --param split_prep=1 > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
f=$(find $O/p -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
r = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for x in r:
    d[x['Kernel_Name'][:40] + ' g' + x['Grid_Size_X']].append(int(x['End_Timestamp']) - int(x['Start_Timestamp']))
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    if len(v) >= 10: print(k, len(v), sorted(v)[len(v) // 2])
PY
