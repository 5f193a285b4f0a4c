#!/bin/bash
# Round 4: keyrank parity tests, then the config-4 leg with keyrank on / off
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r04kr
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "keyrank or full_size_config4 or rank_small_grid or config4_2m" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
i=0
for v in "" "--c4-param keyrank=0"; do
  i=$((i+1))
  timeout -k 10 300 python3 bench.py --config4-only --no-cpu --no-pmc $v > $O/v$i.json 2> $O/v$i.err || { echo "variant $v failed"; tail -5 $O/v$i.err; exit 1; }
  python3 - "$O/v$i.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("config4", d)
print(sys.argv[2], {k: c.get(k) for k in ("ms_per_step", "parity", "host_call_ms_per_step")}, c.get("candidate_sort"))
print("  stages", c.get("stages_ms"))
PY
done
