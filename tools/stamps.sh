#!/bin/bash
# chain phase stamps at a few settings (diagnostic)
export TMPDIR=/tmp
CFGS=${CFGS:-512,3 256,3 0,4}
for cfg in $CFGS; do
  set -- ${cfg//,/ }
  timeout -k 10 120 python bench.py --no-cpu --no-pmc --no-config3 --no-config4 --steps 10 --chain-stamps --chain-warm $1 --chain-passes $2 > gpurun_out/st.log 2>&1 || { tail -5 gpurun_out/st.log; exit 1; }
  tail -1 gpurun_out/st.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('warm=$1 P=$2', round(d['ms_per_step'],4), d['kernels_ms']['chain']['ms'], d['chain_last_batch'], {k: (v[0] if isinstance(v, list) else v) for k, v in d['chain_phases_ns'].items()})"
done
