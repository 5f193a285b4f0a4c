#!/bin/bash
# config-3 time split: per-part timing (synchronised), with and without the enqueue thread pool
export TMPDIR=/tmp
mkdir -p gpurun_out
for extra in "--c3-threads 1" "--c3-threads 0"; do
  timeout -k 10 200 python bench.py --config3-only --no-cpu --no-pmc $extra > gpurun_out/c3p.log 2>&1
  rc=$?; echo "[c3 $extra] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/c3p.log; exit $rc; fi
  tail -1 gpurun_out/c3p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('config3', d); print(round(c['ms_per_step'],3), c['value'], c['parts_ms_per_step'])"
done
