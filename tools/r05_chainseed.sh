#!/bin/bash
# Round 5: chain parity, then level seeds (default) against none, with chain phase stamps
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r05seed
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "golden or fresh or variants or repeated or full_size or depletion or chain or config4 or small_queue" > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do for v in default noseed; do
  if [ "$v" = default ]; then L=""; else L="$GRAFT_REPO_ROOT/adlb_amd/variants/libadlbq_$v.so"; fi
  ADLBQ_LIB=$L timeout -k 10 300 python3 bench.py --no-cpu --no-host-path --no-config3 --no-config4 --no-config5 --no-wide --no-pmc --chain-stamps > $O/$v.$rep.json 2> $O/$v.$rep.err || { echo "$v failed"; tail -5 $O/$v.$rep.err; exit 1; }
  python3 - "$O/$v.$rep.json" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {s: v["ms"] for s, v in d["kernels_ms"].items()}
ph = d.get("chain_phases_ns") or {}
print(f"{sys.argv[2]:8s} ms/step {d['ms_per_step']:.4f} parity {d['parity']} chain {k.get('chain')} rounds {d['chain_last_batch']['rounds']} ph1 {ph.get('phase1')} ph2 {ph.get('phase2')} ph3 {ph.get('phase3')} end {ph.get('end_abs')}")
PY
done; done
