#!/bin/bash
# chain segment / warm-up / passes sweep on the metric leg (phase stamps), parity first per variant
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in s128 s64; do
  ADLBQ_LIB=$PWD/adlb_amd/libadlbq_$lib.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "golden or c2_ or c4_ or fixup or chain" > gpurun_out/sw_par_$lib.log 2>&1
  rc=$?; echo "[parity $lib] rc=$rc $(tail -1 gpurun_out/sw_par_$lib.log)"
  if [ $rc -ge 124 ]; then exit $rc; fi
done
for cfg in "libadlbq 512 3" "libadlbq_s128 256 3" "libadlbq_s128 384 3" "libadlbq_s128 512 3" "libadlbq_s128 256 2" "libadlbq_s64 192 3" "libadlbq_s64 256 3" "libadlbq_s64 384 3" "libadlbq_s64 256 4"; do
  set -- $cfg
  ADLBQ_LIB=$PWD/adlb_amd/$1.so timeout -k 10 120 python bench.py --no-cpu --no-pmc --no-config3 --no-config4 --no-config5 --steps 20 --chain-stamps --chain-warm $2 --chain-passes $3 > gpurun_out/sw.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$cfg rc=$rc"; tail -3 gpurun_out/sw.log; if [ $rc -ge 124 ]; then exit $rc; fi; continue; fi
  tail -1 gpurun_out/sw.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$cfg', round(d['ms_per_step'],4), d['kernels_ms']['chain']['ms'], d['chain_last_batch'], {k: (v[0] if isinstance(v, list) else v) for k, v in d['chain_phases_ns'].items()})"
done
