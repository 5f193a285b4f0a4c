#!/bin/bash
# Round-6 final evidence, part A: every GPU test + smoke, the one-Reserve latency, the driver's bench
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r06
mkdir -p $O
bash tools/r06.sh tests || exit 1
timeout -k 10 200 python3 tools/r05_one.py > $O/one.txt 2>&1 || exit 1
grep -E "R=1|one_b" $O/one.txt
bash tools/r06.sh bench
