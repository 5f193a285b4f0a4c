#!/bin/bash
# Round 5: the config-5 leg three times (run-to-run spread)
export TMPDIR=/tmp
for i in 1 2 3; do
  timeout -k 10 200 python3 bench.py --config5-only --no-pmc --no-cpu > gpurun_out/c5r.json 2> gpurun_out/c5r.err || { tail -5 gpurun_out/c5r.err; exit 1; }
  python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/c5r.json").read().strip().splitlines()[-1])
c = d.get("config5", d)
print(c.get("value"), c.get("seconds"), c.get("parity"))
PY
done
