#!/bin/bash
# config-4 leg with 0, 1, 2 prefix-round launches after round 0 of the ordered choice
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 3 4 2; do
  timeout -k 10 200 python bench.py --no-cpu --no-pmc --config4-only --c4-chain-rounds $k > gpurun_out/c4k$k.log 2>&1 || { tail -5 gpurun_out/c4k$k.log; exit 1; }
  tail -1 gpurun_out/c4k$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['config4']; print('rounds $k', round(d['ms_per_step'],4), '%.3g'%d['value'], d['stages_ms']['chain'])"
done
