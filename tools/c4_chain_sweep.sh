# config-4 chain: parity of the chain variants, then the leg per pass-1 guess with per-batch counters
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "config4 or repeated" -x -v --timeout 180 --timeout-method thread > gpurun_out/gpu_c4.log 2>&1 || exit 1
for g in 1 0; do
  timeout -k 10 120 python bench.py --config4-only --no-cpu --no-pmc --c4-steps 8 --c4-chain-stats --c4-chain-guess $g > gpurun_out/c4_g$g.log 2>&1 || exit 1
done
