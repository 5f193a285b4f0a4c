#!/bin/bash
# Round 5: rocprofv3 kernel statistics of the config-5 leg (SURVEY §8(d) shape, a shorter stream).
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r05c5
rm -rf $O; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 bench.py --config5-only --c5-events ${C5_EVENTS:-2000000} $C5_EXTRA > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
f=$(find $O/p -name "*kernel_stats.csv" | head -1)
cp $f $O/kernel_stats.csv
head -25 $O/kernel_stats.csv | cut -c1-150
