#!/bin/bash
# Round 3: the cross-process steal test, the steal tests, then the default bench (parity gates).
export TMPDIR=/tmp
mkdir -p gpurun_out/r3a
timeout -k 10 300 python -u -m pytest tests/test_gpu_steal_mp.py tests/test_gpu_steal.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r3a/tests.log 2>&1 || { tail -60 gpurun_out/r3a/tests.log; exit 1; }
tail -3 gpurun_out/r3a/tests.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3a/bench.log 2> gpurun_out/r3a/bench.err || { tail -20 gpurun_out/r3a/bench.err; exit 1; }
tail -1 gpurun_out/r3a/bench.log | cut -c1-4000
