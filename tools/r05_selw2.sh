#!/bin/bash
# Round 5: pass-2 stamps, one wave (select_wave=1) against four waves (0).
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r05selw2
mkdir -p $O
for rep in 1 2; do
for v in 1 0; do
  timeout -k 10 300 python3 bench.py --no-cpu --no-host-path --no-config3 --no-config4 --no-config5 --no-wide --no-pmc \
    --param select_wave=$v --kernel-stamps $EXTRA > $O/w$v.$rep.json 2> $O/w$v.$rep.err || { echo "bench $v failed"; tail -5 $O/w$v.$rep.err; exit 1; }
  python3 - "$O/w$v.$rep.json" "w$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {s: v["ms"] for s, v in d["kernels_ms"].items()}
print(f"{sys.argv[2]:6s} ms/step {d['ms_per_step']:.4f} parity {d['parity']} kernels {k}")
if d.get("chain_phases_ns"): print("   stamps", {w: d["chain_phases_ns"][w] for w in ("hist", "sel") if w in d["chain_phases_ns"]})
PY
done
done
