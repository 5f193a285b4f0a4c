#!/bin/bash
# config-4 parity (every config-4 exact test), then a HIP API + kernel trace of the config-4 leg
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $R/gpurun_out/p4.log 2>&1
rc=$?; echo "[parity] rc=$rc $(tail -1 $R/gpurun_out/p4.log)"
if [ $rc -ne 0 ]; then tail -40 $R/gpurun_out/p4.log; exit 1; fi
cd /tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $R/gpurun_out/c4trace -o c4 -- python3 $R/bench.py --config4-only --no-pmc --no-cpu > $R/gpurun_out/c4trace.json 2> $R/gpurun_out/c4trace.err
rc=$?; echo "[trace] rc=$rc"
find $R/gpurun_out/c4trace -name '*stats.csv' | head
tail -1 $R/gpurun_out/c4trace.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read())['config4']; print(d['ms_per_step'], '%.3g'%d['value'], d['host_call_ms_per_step'], d['candidate_sort'], d['stages_ms'])"
