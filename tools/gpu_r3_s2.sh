#!/bin/bash
# Round 3, session 2: parity tests, metric variants, config-3/4 traces.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s2
mkdir -p $O
( while sleep 20; do echo "hb $(date +%s)" >> $O/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/parity.log 2>&1
rc=$?
tail -5 $O/parity.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/parity.log | head -30; exit 1; fi
VARIANTS_FILE=tools/var_gap.txt UBENCH=1 bash tools/gpu_r3_prof.sh s2 || exit 1
bash tools/gpu_r3_legs.sh s2 c4 c4nd c3 || exit 1
