#!/bin/bash
# Round 5: one-wave pass 2 (select_wave=1, default) against the four-wave kernel, parity first.
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r05selw
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "golden or fresh or variants or repeated or full_size or small_queue or dead_pages or depletion" > $O/tests.log 2>&1 \
  || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for rep in 1 2; do
for v in 1 0; do
  timeout -k 10 300 python3 bench.py --no-cpu --no-host-path --no-config3 --no-config4 --no-config5 --no-wide --no-pmc \
    --param select_wave=$v $EXTRA > $O/w$v.$rep.json 2> $O/w$v.$rep.err || { echo "bench $v failed"; tail -5 $O/w$v.$rep.err; exit 1; }
  python3 - "$O/w$v.$rep.json" "w$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = {s: v["ms"] for s, v in d["kernels_ms"].items()}
print(f"{sys.argv[2]:6s} ms/step {d['ms_per_step']:.4f} parity {d['parity']} kernels {k}")
PY
done
done
