#!/bin/bash
# Round 4: the metric leg under adlbq_set_param variants (each "name=v,name=v"), one line each:
#   bash tools/r04_variants.sh "fold_thresholds=0,fuse_rank=0" "fold_thresholds=1" ...
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r04v
mkdir -p $O
python -c "import torch" > /dev/null 2>&1
i=0
for v in "$@"; do
  i=$((i+1))
  P=""
  for kv in $(echo $v | tr ',' ' '); do P="$P --param $kv"; done
  timeout -k 10 300 python3 bench.py --no-cpu --no-host-path --no-config3 --no-config4 --no-config5 --no-wide --no-pmc $EXTRA $P > $O/v$i.json 2> $O/v$i.err || { echo "variant $v failed"; tail -5 $O/v$i.err; exit 1; }
  python3 - "$O/v$i.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {s: v["ms"] for s, v in d["kernels_ms"].items()}
print(f"{sys.argv[2]:40s} ms/step {d['ms_per_step']:.4f} parity {d['parity']} kernels {k} rank_fast {d.get('rank_in_select_last_batch')}")
if d.get("chain_phases_ns"):
    print("   chain phases", d["chain_phases_ns"], "chain", d.get("chain_last_batch"))
PY
done
