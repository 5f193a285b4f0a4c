#!/bin/bash
# parity (host-buffer entry points throughout), then the config-5 leg
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_push.py tests/test_gpu_steal.py -x -q --timeout 300 --timeout-method thread > gpurun_out/p5.log 2>&1
rc=$?; echo "[parity] rc=$rc $(tail -1 gpurun_out/p5.log)"
if [ $rc -ne 0 ]; then tail -40 gpurun_out/p5.log; exit 1; fi
timeout -k 10 300 python bench.py --config5-only --no-pmc --no-cpu > gpurun_out/c5q.log 2>&1 || { tail -5 gpurun_out/c5q.log; exit 1; }
tail -1 gpurun_out/c5q.log | cut -c1-400
