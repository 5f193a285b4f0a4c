#!/bin/bash
# rocprofv3 kernel-trace summaries of the bench legs (GPU box); outputs under gpurun_out/prof_r02/
set -e
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/prof_r02
mkdir -p $O
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/metric -o metric -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --no-pmc --no-config3 --no-config4 --no-config5 > $O/metric_bench.json 2> $O/metric.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o c3 -- python3 $R/bench.py --config3-only --no-pmc --no-cpu > $O/c3_bench.json 2> $O/c3.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o c4 -- python3 $R/bench.py --config4-only --no-pmc --no-cpu > $O/c4_bench.json 2> $O/c4.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o c5 -- python3 $R/bench.py --config5-only --no-pmc --no-cpu > $O/c5_bench.json 2> $O/c5.err
timeout -k 10 400 python3 $R/bench.py > $O/bench_default.json 2> $O/bench_default.err
