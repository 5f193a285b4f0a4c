#!/bin/bash
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/s9
mkdir -p $O
( while sleep 20; do echo "hb $(date +%s)" >> $O/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_steal.py tests/test_gpu_robust.py -x -q --timeout 200 --timeout-method thread -k "full_size_config2 or fixup or variants_vs_oracle or steal_group" > $O/parity.log 2>&1
rc=$?
tail -3 $O/parity.log
if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/parity.log | head -30; exit 1; fi
VARIANTS_FILE=${VF:-tools/var_s8.txt} bash tools/gpu_r3_prof.sh s9 || exit 1
cd $R
timeout -k 10 300 python3 bench.py --config3-only --no-pmc --no-cpu > $O/c3.json 2> $O/c3.err || { echo c3 failed; tail -5 $O/c3.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c3.json').read().strip().splitlines()[-1])['config3'];print('c3 ms',d['ms_per_step'],'parity',d.get('parity'))"
timeout -k 10 300 python3 bench.py --config3-only --no-pmc --no-cpu --c3-parts > $O/c3p.json 2> $O/c3p.err || { echo c3p failed; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c3p.json').read().strip().splitlines()[-1])['config3'];print('c3 parts',d['parts_ms_per_step'])"
