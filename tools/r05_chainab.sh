#!/bin/bash
# Round 5: chain segment / warm-up shapes on the metric leg (variant library + bench flags):
#   bash tools/r05_chainab.sh "default|" "seg128|" "seg128|--chain-warm 384" ...
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r05chain
mkdir -p $O
python -c "import torch" > /dev/null 2>&1
i=0
for rep in 1 2; do
for spec in "$@"; do
  v=${spec%%|*}; fl=${spec#*|}; i=$((i+1))
  if [ "$v" = default ]; then L=""; else L="$GRAFT_REPO_ROOT/adlb_amd/variants/libadlbq_$v.so"; fi
  ADLBQ_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu --no-host-path --no-config3 --no-config4 --no-config5 --no-wide --no-pmc $fl > $O/$i.json 2> $O/$i.err || { echo "variant $spec failed"; tail -5 $O/$i.err; exit 1; }
  python3 - "$O/$i.json" "$spec" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {s: v["ms"] for s, v in d["kernels_ms"].items()}
print(f"{sys.argv[2]:28s} ms/step {d['ms_per_step']:.4f} parity {d['parity']} kernels {k}")
PY
done
done
