#!/bin/bash
# Round-6 evidence on one MI355X (outputs under gpurun_out/r06/):
#   r06.sh tests            every GPU test + smoke
#   r06.sh sel <pytest args> selected GPU tests
#   r06.sh fixed            metric leg at 20 and 100 steps + a kernel trace of the 20-step run (fixed cost per run)
#   r06.sh metric [args]    metric leg only (extra bench arguments appended)
#   r06.sh prof             rocprofv3 kernel stats per bench leg
#   r06.sh bench            the driver's command (--steps 20 --warmup 5)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/r06
mkdir -p $O
( while true; do date +%s > $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
python -c "import torch" > /dev/null 2>&1
PART=${1:-all}
shift
M="--no-cpu --no-pmc --no-host-path --no-config2 --no-config3 --no-config4 --no-config5 --no-wide"
case "$PART" in
sel)
  timeout -k 10 900 python -u -m pytest "$@" -m gpu -v -x --timeout 200 --timeout-method thread > $O/sel.log 2>&1
  rc=$?; echo "[sel] rc=$rc $(tail -1 $O/sel.log)"
  [ $rc -ne 0 ] && grep -E "FAIL|Error|assert" $O/sel.log | head -30
  exit $rc ;;
tests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "[tests] rc=$rc $(tail -1 $O/tests.log)"
  [ $rc -ne 0 ] && grep -E "^FAILED|^ERROR" $O/tests.log | head -30
  if [ $rc -ne 0 ]; then exit $rc; fi
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log ;;
fixed)
  for s in 20 100 20; do
    timeout -k 10 300 python3 bench.py --steps $s --warmup 5 $M "$@" > $O/fixed_$s.json 2> $O/fixed.err || { echo bench failed; tail -5 $O/fixed.err; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('$O/fixed_$s.json').read().strip().splitlines()[-1]); print($s, round(d['ms_per_step'],4), d['timed_region_host_ms'], d['host_submit_ms_per_step'])"
  done
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tl20 -o tl -- python3 $R/bench.py --steps 20 --warmup 5 $M "$@" > $O/tl20.json 2> $O/tl20.err || { echo trace failed; tail -5 $O/tl20.err; exit 1; }
  cd $R
  python3 tools/steps_trace.py $O/tl20 15 20 > $O/tl20_steps.txt
  tail -25 $O/tl20_steps.txt ;;
metric)
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 $M "$@" > $O/metric.json 2> $O/metric.err || { echo bench failed; tail -20 $O/metric.err; exit 1; }
  tail -1 $O/metric.json | cut -c1-2500 ;;
ab)
  # A/B of metric-leg variants: each argument is one variant's extra bench arguments (quoted), run twice
  i=0
  for v in "$@"; do
    for rep in 1 2; do
      timeout -k 10 300 python3 bench.py --steps 100 --warmup 5 $M --chain-stamps $v > $O/ab_$i_$rep.json 2> $O/ab.err || { echo bench failed; tail -5 $O/ab.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/ab_$i_$rep.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],4), {k: v['ms'] for k, v in d['kernels_ms'].items()}, d.get('chain_phases_ns'))"
    done
    i=$((i+1))
  done ;;
prof)
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/metric_prof -o metric -- python3 $R/bench.py --steps 20 --warmup 5 $M > $O/metric_prof.json 2> $O/metric_prof.err || { echo metric prof failed; tail -5 $O/metric_prof.err; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3 -o c3 -- python3 $R/bench.py --config3-only --no-pmc --no-cpu > $O/c3_bench.json 2> $O/c3.err || { echo c3 prof failed; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4 -o c4 -- python3 $R/bench.py --config4-only --no-pmc --no-cpu > $O/c4_bench.json 2> $O/c4.err || { echo c4 prof failed; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o c5 -- python3 $R/bench.py --config5-only --no-pmc --no-cpu --c5-shards 1 --c5-ranks 512 --c5-events 2000000 > $O/c5_bench.json 2> $O/c5.err || { echo c5 prof failed; exit 1; }
  cd $R ;;
bench)
  timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 "$@" > $O/bench.json 2> $O/bench.err || { echo bench failed; tail -20 $O/bench.err; exit 1; }
  tail -1 $O/bench.json | cut -c1-3000 ;;
*)
  echo "unknown part $PART"; exit 2 ;;
esac
