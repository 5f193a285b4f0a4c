#!/bin/bash
# config-4 leg with the ordered choice's per-batch counters
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --no-cpu --no-pmc --config4-only --c4-chain-stats > gpurun_out/c4cs.log 2>&1 || { tail -5 gpurun_out/c4cs.log; exit 1; }
tail -1 gpurun_out/c4cs.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['config4']; print(d['ms_per_step'], d['chain_per_batch'])"
