#!/bin/bash
# Round 4: config-4 k_targeted_idx with parts skipped (targeted_diag 1: lists only, 2: + cache fill; wrong results)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r04tdiag
mkdir -p $O
for d in ${DIAGS:-0 1 2}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/p$d -o run -- python3 bench.py --config4-only --no-cpu --no-pmc --c4-param targeted_diag=$d > $O/b$d.json 2> $O/b$d.err || { tail -5 $O/b$d.err; exit 1; }
  f=$(find $O/p$d -name "*kernel_trace.csv" | head -1)
  python3 - "$f" $d <<'PY'
import csv, sys
r = [int(x['End_Timestamp']) - int(x['Start_Timestamp']) for x in csv.DictReader(open(sys.argv[1])) if 'k_targeted_idx' in x['Kernel_Name']]
print('targeted_diag', sys.argv[2], sorted(r)[len(r) // 2], r[-8:])
PY
done
