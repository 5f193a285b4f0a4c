#!/bin/bash
# Round 4: parity (all T > 8 and golden cases), then the config-4 leg
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r04prep
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "${KEXPR:-golden or fresh or keyrank or config4 or t64 or c4}" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 bench.py --config4-only --no-cpu --no-pmc > $O/c4.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 1; }
python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d.get('config4',d); print(c.get('ms_per_step'), c.get('parity'), c.get('host_call_ms_per_step'), c.get('stages_ms'))" $O/c4.json
