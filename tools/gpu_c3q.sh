#!/bin/bash
# steal parity, then the config-3 leg
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_steal.py tests/test_gpu_server.py -x -q --timeout 300 --timeout-method thread > gpurun_out/st.log 2>&1
rc=$?; echo "[steal] rc=$rc $(tail -1 gpurun_out/st.log)"
if [ $rc -ne 0 ]; then tail -40 gpurun_out/st.log; exit 1; fi
timeout -k 10 300 python bench.py --config3-only --no-pmc --no-cpu > gpurun_out/c3q.log 2>&1 || { tail -5 gpurun_out/c3q.log; exit 1; }
tail -1 gpurun_out/c3q.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['config3']; print(d['ms_per_step'], '%.3g'%d['value'], d.get('parts_ms_per_step'))"
