#!/bin/bash
# Round 3: the steal-group / server tests again (after the multi-shard settle), then the profiles and the default bench.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03
mkdir -p $O
( while true; do date +%s > $O/heartbeat_b; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
python -c "import torch" > /dev/null 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_steal.py tests/test_gpu_server.py -v --timeout 200 --timeout-method thread > $O/tests_steal.log 2>&1
rc=$?; echo "[steal/server tests] rc=$rc $(tail -1 $O/tests_steal.log)"
if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $O/tests_steal.log | head -20; exit 1; fi
bash tools/final_r03.sh prof
