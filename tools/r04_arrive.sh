#!/bin/bash
# Round 4: pass-1 chunk sums by the chunk's last page (hist_arrive): parity tests, then A/B on the metric,
# config 3 and config 4 legs
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r04arr
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_group.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for a in 1 0 1 0; do
  timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-host-path --no-config5 --no-wide --param hist_arrive=$a --c3-param hist_arrive=$a --c4-param hist_arrive=$a > $O/b$a.json 2> $O/b$a.err || { tail -5 $O/b$a.err; exit 1; }
  python3 - $O/b$a.json $a <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('hist_arrive', sys.argv[2], 'metric', round(d['ms_per_step'], 4), 'c3', round(d['config3']['ms_per_step'], 4), 'c4', round(d['config4']['ms_per_step'], 4), d['config4']['stages_ms'].get('hist'), d['parity'] if 'parity' in d else '', d['config3'].get('parity'), d['config4'].get('parity'))
PY
done
