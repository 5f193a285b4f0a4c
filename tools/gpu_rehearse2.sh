#!/bin/bash
# Rehearse bench.py's two-rank path on one GPU (gloo, both ranks on device 0): code paths only.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/rh2
mkdir -p $O
( while true; do date +%s > $O/heartbeat; sleep 20; done ) &
HB=$!
trap "kill $HB" EXIT
export ADLB_BENCH_REHEARSE=1
timeout -k 10 700 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --config5-only > $O/bench2.json 2> $O/bench2.err
rc=$?; echo "rc=$rc"; tail -1 $O/bench2.json | cut -c1-1500; if [ $rc -ne 0 ]; then grep -v "^\s*$" $O/bench2.err | tail -30; fi
