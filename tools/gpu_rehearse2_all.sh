#!/bin/bash
# Rehearse every bench.py leg at two ranks on one GPU (gloo, both ranks on device 0): code paths only.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rh2
mkdir -p $O
( while true; do date +%s > $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
export ADLB_BENCH_REHEARSE=1
timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --no-pmc --no-host-path > $O/bench2all.json 2> $O/bench2all.err
rc=$?; echo "rc=$rc"
python3 - $O/bench2all.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("metric", d.get("value"), d.get("ms_per_step"), d.get("parity"), d.get("n_gpus"))
for k in ("config3", "config4", "config5", "wide_types"):
    c = d.get(k, {})
    print(k, {x: c.get(x) for x in ("value", "ms_per_step", "parity", "error")})
PY
if [ $rc -ne 0 ]; then grep -v "^\s*$" $O/bench2all.err | tail -30; fi
exit $rc
