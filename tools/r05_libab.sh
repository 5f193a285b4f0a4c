#!/bin/bash
# Round 5: the metric leg with experimental library builds (tools/build_variant.sh), alternated:
#   bash tools/r05_libab.sh default nolump v0 ...      (default = adlb_amd/libadlbq.so)
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r05ab
mkdir -p $O
python -c "import torch" > /dev/null 2>&1
for rep in 1 2; do
for v in "$@"; do
  if [ "$v" = default ]; then L=""; else L="$GRAFT_REPO_ROOT/adlb_amd/variants/libadlbq_$v.so"; fi
  ADLBQ_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu --no-host-path --no-config3 --no-config4 --no-config5 --no-wide --no-pmc $EXTRA > $O/$v.$rep.json 2> $O/$v.$rep.err || { echo "variant $v failed"; tail -5 $O/$v.$rep.err; exit 1; }
  python3 - "$O/$v.$rep.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {s: v["ms"] for s, v in d["kernels_ms"].items()}
print(f"{sys.argv[2]:12s} ms/step {d['ms_per_step']:.4f} parity {d['parity']} kernels {k}")
if d.get("chain_phases_ns"): print("   stamps", {w: d["chain_phases_ns"][w] for w in ("hist", "sel") if w in d["chain_phases_ns"]})
PY
done
done
