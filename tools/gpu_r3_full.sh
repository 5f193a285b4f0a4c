#!/bin/bash
# Round 3: every GPU test, smoke, then the default bench (parity gates on every leg).
export TMPDIR=/tmp
mkdir -p gpurun_out/r3full
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3full/tests.log 2>&1 || { grep -E "FAIL|ERROR|Error" gpurun_out/r3full/tests.log | tail -40; tail -60 gpurun_out/r3full/tests.log; exit 1; }
tail -3 gpurun_out/r3full/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3full/smoke.log 2>&1 || { cat gpurun_out/r3full/smoke.log; exit 1; }
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3full/bench.log 2> gpurun_out/r3full/bench.err || { tail -20 gpurun_out/r3full/bench.err; exit 1; }
tail -1 gpurun_out/r3full/bench.log | cut -c1-6000
timeout -k 10 60 tools/ubench_scan > gpurun_out/r3full/ubench_scan.txt 2>&1 || true
cat gpurun_out/r3full/ubench_scan.txt
