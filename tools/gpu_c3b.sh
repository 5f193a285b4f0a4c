#!/bin/bash
# parity (gpu parity + steal), then config 3 / metric / config 4 legs
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_steal.py tests/test_gpu_push.py -x -q --timeout 120 --timeout-method thread > gpurun_out/p.log 2>&1
rc=$?; echo "[parity] rc=$rc $(tail -1 gpurun_out/p.log)"
if [ $rc -ne 0 ]; then tail -40 gpurun_out/p.log; exit 1; fi
for extra in "--config4-only" "--config5-only" "--config3-only" "--no-config3 --no-config4 --no-config5"; do
  timeout -k 10 200 python bench.py --no-cpu --no-pmc $extra > gpurun_out/b.log 2>&1
  rc=$?; echo "[$extra] rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/b.log; exit $rc; fi
  tail -1 gpurun_out/b.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
for k in ('config3','config4','config5'):
    if k in d: c=d[k]; print(k, round(c.get('ms_per_step',0),3), '%.3g'%c['value'], c.get('parts_ms_per_step'), c.get('host_call_ms_per_step'), c.get('parity_with_oracle'))
if 'metric' in d: print('metric', round(d['ms_per_step'],4), '%.4g'%d['value'], d['host_submit_ms_per_step'])"
done
