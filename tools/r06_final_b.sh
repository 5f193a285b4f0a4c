#!/bin/bash
# Round-6 final evidence, part B: rocprofv3 kernel stats per bench leg, the metric leg's kernel trace
# (20 steps: fixed cost per run), the one-Reserve kernel
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r06
mkdir -p $O
bash tools/r06.sh prof || exit 1
bash tools/r06.sh fixed || exit 1
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/one_prof -o one -- python3 $GRAFT_REPO_ROOT/tools/r05_one.py > $O/one_prof.txt 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 bench.py --units 1000000 --steps 20 --warmup 5 --no-cpu --no-pmc --no-host-path --no-config2 --no-config3 --no-config4 --no-config5 --no-wide > $O/m1m.json 2> $O/m1m.err || exit 1
python3 -c "import json; d=json.loads(open('$O/m1m.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['parity'], {k: v['ms'] for k, v in d['kernels_ms'].items()}, d.get('chain_last_batch'), d.get('candidates_last_batch'))"
