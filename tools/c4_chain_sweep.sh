# config-4 chain: parity with warm-up on the wide variant, then the leg per warm-up / pass count
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "config4 or repeated" -x -v --timeout 180 --timeout-method thread > gpurun_out/gpu_c4.log 2>&1 || exit 1
for wk in "0 8" "256 8" "512 8" "512 4" "256 4"; do
  set -- $wk
  timeout -k 10 120 python bench.py --config4-only --no-cpu --no-pmc --c4-steps 10 --c4-chain-warm $1 --c4-chain-passes $2 > gpurun_out/c4_w$1_k$2.log 2>&1 || exit 1
done
