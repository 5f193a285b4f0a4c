#!/bin/bash
# round-end evidence: every GPU test, smoke, rocprof kernel stats per bench leg, default bench
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $R/gpurun_out/final_tests.log 2>&1
rc=$?; echo "[tests] rc=$rc $(tail -1 $R/gpurun_out/final_tests.log)"
if [ $rc -ge 124 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $R/gpurun_out/final_smoke.log 2>&1 || { echo smoke failed; tail -5 $R/gpurun_out/final_smoke.log; exit 1; }
tail -1 $R/gpurun_out/final_smoke.log
bash tools/profile_r02.sh || { echo "profile failed"; exit 1; }
python tools/step_timeline.py $R/gpurun_out/prof_r02/metric > $R/gpurun_out/prof_r02/step_timeline.txt 2>&1
tail -1 $R/gpurun_out/prof_r02/bench_default.json | cut -c1-400
