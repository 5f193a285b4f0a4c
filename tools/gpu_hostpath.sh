#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --no-cpu --no-pmc --no-config3 --no-config4 --no-config5 > gpurun_out/hp.log 2>&1 || { tail -5 gpurun_out/hp.log; exit 1; }
tail -1 gpurun_out/hp.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], '%.4g'%d['value'], d['host_buffer_path'])"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "golden or c2_n200k or exhaust" -q -rs --timeout 250 --timeout-method thread > gpurun_out/push_tests.log 2>&1
echo "[tests] rc=$? $(tail -1 gpurun_out/push_tests.log)"; grep SKIP gpurun_out/push_tests.log | head
