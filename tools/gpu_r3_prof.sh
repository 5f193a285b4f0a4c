#!/bin/bash
# Round 3: metric-leg kernel timelines (rocprofv3 kernel trace), one run per variant.
# usage: [VARIANTS_FILE=f] tools/gpu_r3_prof.sh <tag> [extra bench args...]
# variants: lines "name:bench args" (default: base only)
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
if [ -n "$VARIANTS_FILE" ]; then mapfile -t VARIANTS < $VARIANTS_FILE; else VARIANTS=("base:"); fi
( while sleep 20; do echo "hb $(date +%s)" >> $O/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp
timeout -k 10 200 python3 -c "import torch; print('torch', torch.__version__, torch.cuda.is_available())" || exit 1
if [ -x $R/tools/ubench_scan ] && [ -n "$UBENCH" ]; then timeout -k 10 120 $R/tools/ubench_scan > $O/ubench_scan.txt 2>&1; cat $O/ubench_scan.txt; fi
for v in "${VARIANTS[@]}"; do
    n=${v%%:*}; a=${v#*:}
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o $n -- python3 $R/bench.py --steps 30 --warmup 5 --no-cpu --no-pmc --no-config3 --no-config4 --no-config5 --no-host-path $a "$@" > $O/$n.json 2> $O/$n.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "variant $n failed rc=$rc"; tail -20 $O/$n.err; exit 1; fi
    python3 $R/tools/step_timeline.py $O/$n > $O/$n.timeline.txt
    echo "== $n"; cat $O/$n.timeline.txt
    python3 -c "import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);print('ms_per_step',d['ms_per_step'],'parity',d.get('parity'),'chain',d.get('chain_last_batch'))"
done
