#!/bin/bash
# Round 4: the config-4 leg under variants (each a quoted list of bench.py arguments), one line each
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r04c4
mkdir -p $O
python -c "import torch" > /dev/null 2>&1
i=0
for v in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python3 bench.py --config4-only --no-cpu --no-pmc $v > $O/v$i.json 2> $O/v$i.err || { echo "variant $v failed"; tail -5 $O/v$i.err; exit 1; }
  python3 - "$O/v$i.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = d.get("config4", d)
print(sys.argv[2], {k: c.get(k) for k in ("ms_per_step", "parity")}, "chain", (c.get("stages_ms") or {}).get("chain"))
PY
done
