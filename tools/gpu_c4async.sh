#!/bin/bash
# sync-free candidate sort: config-4 parity, then the config-4 leg (async on / off)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "c4 or golden or sort or c2_t64" > gpurun_out/c4a_par.log 2>&1
rc=$?; echo "[parity] rc=$rc $(tail -1 gpurun_out/c4a_par.log)"
if [ $rc -ne 0 ]; then tail -30 gpurun_out/c4a_par.log; exit 1; fi
for a in 1 0; do
  timeout -k 10 200 python bench.py --config4-only --no-cpu --no-pmc --c4-segsort-async $a > gpurun_out/c4a.log 2>&1
  rc=$?; echo "[c4 async=$a] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/c4a.log; exit $rc; fi
  tail -1 gpurun_out/c4a.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('config4', d); c.pop('workload',None); print(json.dumps(c)[:900])"
done
