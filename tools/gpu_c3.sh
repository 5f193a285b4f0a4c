#!/bin/bash
# steal-round parity (incl. the export gathered from the last batch), then the config-3 leg and its parts
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_steal.py -x -q --timeout 120 --timeout-method thread > gpurun_out/c3_par.log 2>&1
rc=$?; echo "[steal parity] rc=$rc $(tail -1 gpurun_out/c3_par.log)"
if [ $rc -ne 0 ]; then tail -40 gpurun_out/c3_par.log; exit 1; fi
for extra in "" "--c3-parts"; do
  timeout -k 10 200 python bench.py --config3-only --no-cpu --no-pmc $extra > gpurun_out/c3.log 2>&1
  rc=$?; echo "[c3 $extra] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/c3.log; exit $rc; fi
  tail -1 gpurun_out/c3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d.get('config3', d); print(round(c['ms_per_step'],3), c['value'], c['parts_ms_per_step'], c['steal_check'])"
done
