#!/bin/bash
# Round-5 evidence on one MI355X (outputs under gpurun_out/r05/):
#   final_r05.sh tests   every GPU test + smoke
#   final_r05.sh sel <pytest arguments>   selected GPU tests
#   final_r05.sh prof    rocprofv3 kernel stats per bench leg + the step timeline
#   final_r05.sh bench   the default bench
#   final_r05.sh all     tests, prof, bench
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05
mkdir -p $O
( while true; do date +%s > $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
python -c "import torch" > /dev/null 2>&1
PART=${1:-all}
if [ "$PART" = "sel" ]; then
  shift
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -v -x --timeout 200 --timeout-method thread > $O/sel.log 2>&1
  rc=$?; echo "[sel] rc=$rc $(tail -1 $O/sel.log)"
  [ $rc -ne 0 ] && grep -E "FAIL|Error|assert" $O/sel.log | head -30
  exit $rc
fi
if [ "$PART" = "tests" ] || [ "$PART" = "all" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "[tests] rc=$rc $(tail -1 $O/tests.log)"
  [ $rc -ne 0 ] && grep -E "^FAILED|^ERROR" $O/tests.log | head -30
  if [ $rc -ge 124 ]; then exit $rc; fi
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
  [ "$PART" = "tests" ] && exit $rc
fi
if [ "$PART" = "prof" ] || [ "$PART" = "all" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/metric -o metric -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu --no-pmc --no-host-path --no-config3 --no-config4 --no-config5 --no-wide > $O/metric_bench.json 2> $O/metric.err || { echo metric prof failed; tail -5 $O/metric.err; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o c3 -- python3 $R/bench.py --config3-only --no-pmc --no-cpu > $O/c3_bench.json 2> $O/c3.err || { echo c3 prof failed; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o c4 -- python3 $R/bench.py --config4-only --no-pmc --no-cpu > $O/c4_bench.json 2> $O/c4.err || { echo c4 prof failed; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o c5 -- python3 $R/bench.py --config5-only --no-pmc --no-cpu --c5-shards 1 --c5-ranks 512 --c5-events 2000000 > $O/c5_bench.json 2> $O/c5.err || { echo c5 prof failed; exit 1; }
  cd $R
  python tools/step_timeline.py $O/metric > $O/step_timeline.txt 2>&1
fi
if [ "$PART" = "bench" ] || [ "$PART" = "all" ]; then
  timeout -k 10 600 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { echo bench failed; tail -20 $O/bench_default.err; exit 1; }
  tail -1 $O/bench_default.json | cut -c1-3000
fi
if [ "$PART" = "metric" ]; then
  timeout -k 10 300 python3 bench.py --no-cpu --no-host-path --no-config3 --no-config4 --no-config5 --no-wide > $O/metric_only.json 2> $O/metric_only.err || { echo bench failed; tail -20 $O/metric_only.err; exit 1; }
  tail -1 $O/metric_only.json | cut -c1-1500
fi
