#!/bin/bash
# Quick GPU iteration: parity tests, then the metric leg and the config-4 leg (no PMC / CPU legs).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/q_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/q_tests.log; exit 1; }
tail -3 gpurun_out/q_tests.log
timeout -k 10 200 python bench.py --no-cpu --no-pmc --no-config3 --no-config4 $BENCH_ARGS > gpurun_out/q_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/q_bench.log; exit 1; }
tail -1 gpurun_out/q_bench.log | cut -c1-1500
timeout -k 10 200 python bench.py --config4-only --no-cpu --no-pmc --c4-chain-stats $C4_ARGS > gpurun_out/q_c4.log 2>&1 || { echo "c4 failed"; tail -20 gpurun_out/q_c4.log; exit 1; }
tail -1 gpurun_out/q_c4.log | cut -c1-3000
