# config-4 leg per chain pass count (results never depend on it)
mkdir -p gpurun_out
for k in 4 8 12 16 24; do
  timeout -k 10 120 python bench.py --config4-only --no-cpu --no-pmc --c4-steps 10 --c4-chain-passes $k > gpurun_out/c4_k$k.log 2>&1 || exit 1
done
