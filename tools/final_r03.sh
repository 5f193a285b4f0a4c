#!/bin/bash
# Round-3 evidence on one MI355X: every GPU test, smoke, rocprof kernel stats per
# bench leg, the step timeline, then the default bench.  Outputs under gpurun_out/r03/.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03
mkdir -p $O
( while true; do date +%s > $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
python -c "import torch" > /dev/null 2>&1
PART=${1:-all}
if [ "$PART" != "prof" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "[tests] rc=$rc $(tail -1 $O/tests.log)"
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
[ "$PART" = "tests" ] && exit 0
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/metric -o metric -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --no-pmc --no-host-path --no-config3 --no-config4 --no-config5 > $O/metric_bench.json 2> $O/metric.err || { echo metric prof failed; tail -5 $O/metric.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o c3 -- python3 $R/bench.py --config3-only --no-pmc --no-cpu > $O/c3_bench.json 2> $O/c3.err || { echo c3 prof failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o c4 -- python3 $R/bench.py --config4-only --no-pmc --no-cpu > $O/c4_bench.json 2> $O/c4.err || { echo c4 prof failed; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o c5 -- python3 $R/bench.py --config5-only --no-pmc --no-cpu > $O/c5_bench.json 2> $O/c5.err || { echo c5 prof failed; exit 1; }
cd $R
python tools/step_timeline.py $O/metric > $O/step_timeline.txt 2>&1
timeout -k 10 600 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo bench failed; tail -20 $O/bench_default.err; exit 1; }
tail -1 $O/bench_default.json | cut -c1-3000
