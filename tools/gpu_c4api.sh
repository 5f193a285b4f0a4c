#!/bin/bash
# config-4 leg under a HIP API trace: which host calls take the step's host time
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c4api
mkdir -p $O
( while true; do date +%s > $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
python -c "import torch" > /dev/null 2>&1
cd /tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $O/t -o c4 -- python3 $R/bench.py --config4-only --no-pmc --no-cpu > $O/c4.json 2> $O/c4.err || { echo failed; tail -5 $O/c4.err; exit 1; }
ls $O/t
