#!/bin/bash
# Round-3 baseline: GPU tests, smoke, and the driver's default bench command.
export TMPDIR=/tmp
mkdir -p gpurun_out/r3base
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3base/gpu_tests.log 2>&1 || { tail -30 gpurun_out/r3base/gpu_tests.log; exit 1; }
tail -3 gpurun_out/r3base/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3base/smoke.log 2>&1 || exit 1
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3base/bench.log 2> gpurun_out/r3base/bench.err || { tail -20 gpurun_out/r3base/bench.err; exit 1; }
tail -1 gpurun_out/r3base/bench.log | cut -c1-3000

