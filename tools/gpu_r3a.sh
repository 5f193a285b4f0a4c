#!/bin/bash
# tests (parity incl. put-side FIFO + push), mix probes, bench, stamps; stop only on hangs/crashes
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stop after $name"; exit $rc; fi
  return 0
}
run tests 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
tail -5 gpurun_out/tests.log
for cfg in "6 2 100 2000 120000" "7 3 150 2000 250000" "10 4 200 1000 150000"; do
  set -- $cfg
  run mix_$2_$5 120 /opt/conda/bin/mpirun -np $1 tests/apps/adlb_mix -nservers $2 -n $3 -len $4 -hi $5
  grep -E "^(server|adlb_mix)" gpurun_out/mix_$2_$5.log
done
run bench 300 python bench.py
tail -1 gpurun_out/bench.log | cut -c1-2500
run stamps 200 python bench.py --no-cpu --no-pmc --no-config3 --no-config4 --steps 10 --chain-stamps
tail -1 gpurun_out/stamps.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['kernels_ms']['chain'], d['chain_last_batch'], d.get('chain_phases_ns'))"
