#!/bin/bash
# Round 3: every GPU test (new: cross-process steal group, robustness), then the default bench (parity gates).
export TMPDIR=/tmp
mkdir -p gpurun_out/r3b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3b/tests.log 2>&1 || { grep -E "PASS|FAIL|ERROR|Error" gpurun_out/r3b/tests.log | tail -40; tail -60 gpurun_out/r3b/tests.log; exit 1; }
tail -3 gpurun_out/r3b/tests.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3b/bench.log 2> gpurun_out/r3b/bench.err || { tail -20 gpurun_out/r3b/bench.err; exit 1; }
tail -1 gpurun_out/r3b/bench.log | cut -c1-5000
