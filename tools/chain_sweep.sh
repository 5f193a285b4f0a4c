#!/bin/bash
# Ordered-choice parameter sweep on the GPU (metric leg and config-4 leg).
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "chain or fresh or golden or repeated" > gpurun_out/sw_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/sw_tests.log; exit 1; }
tail -2 gpurun_out/sw_tests.log
x() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); d=d.get('config4',d); print(sys.argv[2], round(d['ms_per_step'],4), d.get('kernels_ms',{}).get('chain',{}).get('ms', d.get('stages_ms',{}).get('chain')), d.get('chain_last_batch', [ (b['chain_passes'],b['chain_recomputed'],b['chain_fallback']) for b in d.get('chain_per_batch',[])]))" "$@"; }
for cfg in $C2_CFGS; do
  set -- ${cfg//,/ }
  timeout -k 10 120 python bench.py --no-cpu --no-pmc --no-config3 --no-config4 --steps 10 --chain-warm $1 --chain-passes $2 --chain-rounds $3 > gpurun_out/sw_c2.log 2>&1 || { echo "bench failed $cfg"; tail -5 gpurun_out/sw_c2.log; exit 1; }
  x gpurun_out/sw_c2.log "c2 warm=$1 P=$2 K=$3"
done
for cfg in $C4_CFGS; do
  set -- ${cfg//,/ }
  timeout -k 10 150 python bench.py --config4-only --no-cpu --no-pmc --c4-chain-stats --c4-chain-passes $1 --c4-chain-rounds $2 > gpurun_out/sw_c4.log 2>&1 || { echo "c4 failed $cfg"; tail -5 gpurun_out/sw_c4.log; exit 1; }
  x gpurun_out/sw_c4.log "c4 P=$1 K=$2"
done
if [ -n "$PROF" ]; then
  rm -rf gpurun_out/sw_prof
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sw_prof -o run -- python3 bench.py --no-cpu --no-pmc --no-config3 --no-config4 --no-profile --steps 10 $PROF > gpurun_out/sw_prof.log 2>&1 || { echo "prof failed"; exit 1; }
  python3 - <<'PY'
import csv,glob
f=glob.glob('gpurun_out/sw_prof/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]: print(r['Name'][:60].ljust(60), r['Calls'].rjust(4), round(float(r['AverageNs'])/1000,2))
PY
fi
