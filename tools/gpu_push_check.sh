#!/bin/bash
# push protocol on the GPU: engine goldens + two-core push tests + server replays, then live mix runs
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_push.py tests/test_gpu_server.py "tests/test_gpu_parity.py::test_golden" -x -q --timeout 120 --timeout-method thread > gpurun_out/push_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/push_tests.log; exit 1; }
tail -3 gpurun_out/push_tests.log
for cfg in "6 2 100 2000 120000" "7 3 150 2000 250000" "7 3 150 2000 400000" "10 4 200 1000 150000"; do
  set -- $cfg
  timeout -k 10 120 /opt/conda/bin/mpirun -np $1 tests/apps/adlb_mix -nservers $2 -n $3 -len $4 -hi $5 > gpurun_out/mix_$2_$5.log 2>&1 || { echo "mix $cfg failed"; tail -20 gpurun_out/mix_$2_$5.log; exit 1; }
  echo "== $cfg"; grep -E "^(server|adlb_mix)" gpurun_out/mix_$2_$5.log
done
