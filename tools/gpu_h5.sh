#!/bin/bash
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/h5
mkdir -p $O
( while true; do date +%s > $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "targeted or config4 or c4_ or stream" > $O/parity.log 2>&1
rc=$?; tail -2 $O/parity.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" $O/parity.log | head; exit 1; fi
timeout -k 10 300 python3 bench.py --config4-only --no-pmc --no-cpu > $O/c4.json 2> $O/c4.err || { echo failed; tail -5 $O/c4.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c4.json').read().strip().splitlines()[-1])['config4'];print(d['ms_per_step'],d['parity'],d['host_call_parts_ms'],d['reserve_host_sections_ms'],d['stages_ms'])"
timeout -k 10 300 python3 bench.py --config5-only --no-pmc --no-cpu --c5-procs 0 > $O/c5.json 2> $O/c5.err || { echo c5 failed; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c5.json').read().strip().splitlines()[-1])['config5'];print('c5',d['value'],d['parity'])"
