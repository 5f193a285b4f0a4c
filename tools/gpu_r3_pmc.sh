#!/bin/bash
# Round 3: SQ counters per dispatch of the metric leg's kernels (one PMC pass), heartbeat for the watchdog.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc_$1
shift
mkdir -p $O
( while sleep 20; do echo "hb $(date +%s)" >> $O/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp
timeout -k 10 200 python3 -c "import torch; print(torch.cuda.is_available())" || exit 1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $O/sq -o sq -- python3 $R/bench.py --steps 4 --warmup 2 --no-cpu --no-pmc --no-config3 --no-config4 --no-config5 --no-host-path --no-profile "$@" > $O/sq.json 2> $O/sq.err
echo rc=$?
python3 - $O <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/sq/**/*counter_collection.csv", recursive=True)
if not f: print("no counter csv"); sys.exit(0)
rows = list(csv.DictReader(open(f[0])))
agg = collections.OrderedDict()
for r in rows:
    k = (r["Dispatch_Id"], r["Kernel_Name"][:48])
    agg.setdefault(k, {})[r["Counter_Name"]] = float(r["Counter_Value"])
last = list(agg.items())[-40:]
for (d, n), c in last:
    print(d, n, " ".join(f"{k.replace('SQ_','')}={int(v)}" for k, v in c.items()))
PY
