#!/bin/bash
# golden parity, then the metric leg and the config-4 leg (stage GPU and host times)
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "golden or c4 or unreserve or repeated" > gpurun_out/p.log 2>&1
rc=$?; echo "[parity] rc=$rc $(tail -1 gpurun_out/p.log)"
if [ $rc -ne 0 ]; then tail -40 gpurun_out/p.log; exit 1; fi
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu --no-pmc --no-config3 --no-config4 --no-config5 --no-host-path > gpurun_out/m.log 2>&1 || { tail -5 gpurun_out/m.log; exit 1; }
tail -1 gpurun_out/m.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('metric', d['ms_per_step'], '%.4g'%d['value'])"
timeout -k 10 200 python bench.py --no-cpu --no-pmc --config4-only > gpurun_out/b.log 2>&1 || { tail -5 gpurun_out/b.log; exit 1; }
tail -1 gpurun_out/b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['config4']; print(d['ms_per_step'], '%.3g'%d['value'], d['host_call_ms_per_step'], d['host_call_parts_ms'], d['candidate_sort'], d['stages_ms'], d['stages_host_ms'])"
