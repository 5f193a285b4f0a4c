#!/bin/bash
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c3h2
mkdir -p $O
( while true; do date +%s > $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_robust.py tests/test_gpu_steal.py tests/test_gpu_steal_mp.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $O/tests.log | head; exit 1; fi
timeout -k 10 300 python3 bench.py --config3-only --no-pmc --no-cpu > $O/c3.json 2> $O/c3.err || { echo c3 failed; tail -5 $O/c3.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c3.json').read().strip().splitlines()[-1])['config3'];print('c3',d['ms_per_step'],d['parity'],d['reserve_host_sections_ms_per_step'],d['reserve_host_counts_per_step'])"
