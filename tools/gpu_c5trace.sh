#!/bin/bash
# HIP API + kernel trace of the config-5 leg
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $R/gpurun_out/c5trace -o c5 -- python3 $R/bench.py --config5-only --no-pmc --no-cpu > $R/gpurun_out/c5trace.json 2> $R/gpurun_out/c5trace.err
rc=$?; echo "[trace] rc=$rc"
tail -1 $R/gpurun_out/c5trace.json | cut -c1-600
