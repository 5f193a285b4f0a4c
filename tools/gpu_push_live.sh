#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 150 /opt/conda/bin/mpirun -np 6 tests/apps/adlb_push -n 300 -len 1000 -hi 80000 > gpurun_out/push_live.log 2>&1
echo "[push app] rc=$?"; grep -E "^(server|adlb_push)|\*\*|rc " gpurun_out/push_live.log | head -20
timeout -k 10 300 python -u -m pytest tests/test_gpu_server.py tests/test_gpu_push.py -x -q -rs --timeout 250 --timeout-method thread > gpurun_out/push_tests.log 2>&1
echo "[tests] rc=$? $(tail -1 gpurun_out/push_tests.log)"
