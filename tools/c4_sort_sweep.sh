# config-4 sort paths on the GPU: parity of every path, then the bench leg per path
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "config4 or repeated" -x -v --timeout 180 --timeout-method thread > gpurun_out/gpu_c4.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --config4-only --no-cpu --no-pmc > gpurun_out/c4_merged.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --config4-only --no-cpu --no-pmc --c4-segsort-wide 8192 > gpurun_out/c4_w8192.log 2>&1 || exit 1
