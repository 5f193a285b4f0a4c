#!/bin/bash
# Round 4: rq backpressure by the oldest landed snapshot (default) vs a stream sync: tests, then the metric
# and config-3/4 legs alternated
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r04rq
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "repeated or depletion or stream or put_side or bytes" tests/test_gpu_group.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for a in 0 1 0 1; do
  timeout -k 10 300 python3 bench.py --no-cpu --no-pmc --no-host-path --no-config5 --no-wide --param rq_wait_sync=$a --c3-param rq_wait_sync=$a --c4-param rq_wait_sync=$a > $O/b$a.json 2> $O/b$a.err || { tail -5 $O/b$a.err; exit 1; }
  python3 - $O/b$a.json $a <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('rq_wait_sync', sys.argv[2], 'metric', round(d['ms_per_step'], 4), d['reserve_host_sections_ms_per_step'].get('rq_cap'), 'c3', round(d['config3']['ms_per_step'], 4), 'c4', round(d['config4']['ms_per_step'], 4), d['parity'], d['config3'].get('parity'), d['config4'].get('parity'))
PY
done
