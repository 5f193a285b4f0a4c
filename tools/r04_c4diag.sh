#!/bin/bash
# Round 4: config-4 pass 1 with its flush skipped / loads only (extra diagnostic launch before the real one)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r04c4diag
mkdir -p $O
for d in split; do
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/p$d -o run -- python3 bench.py --config4-only --no-cpu --no-pmc --c4-param split_prep=1 > $O/b$d.json 2> $O/b$d.err || { tail -5 $O/b$d.err; exit 1; }
  f=$(find $O/p$d -name "*kernel_trace.csv" | head -1)
  python3 - "$f" $d <<'PY'
import csv, sys
r = [x for x in csv.DictReader(open(sys.argv[1])) if 'k_prep_hist' in x['Kernel_Name']]
d = [int(x['End_Timestamp']) - int(x['Start_Timestamp']) for x in r]
print(sys.argv[2], 'prep role', d[-16::2], 'pass 1', d[-15::2])
PY
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d.get('config4',d); print(c.get('ms_per_step'), c.get('parity'), c.get('candidate_sort'))" $O/b$d.json
done
