#!/bin/bash
# Round 3: kernel traces of the config-3 and config-4 legs (rocprofv3), heartbeat for the silence watchdog.
# usage: tools/gpu_r3_legs.sh <tag> [c3|c4 ...]
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
TAG=$1; shift
O=$R/gpurun_out/legs_$TAG
mkdir -p $O
( while sleep 20; do echo "hb $(date +%s)" >> $O/heartbeat.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp
for leg in "$@"; do
    case $leg in
        c3) args="--config3-only --no-pmc --no-cpu" ;;
        c3t) args="--config3-only --no-pmc --no-cpu --c3-threads 1" ;;
        c3p) args="--config3-only --no-pmc --no-cpu --c3-parts" ;;
        c4) args="--config4-only --no-pmc --no-cpu" ;;
        c4nd) args="--config4-only --no-pmc --no-cpu --c4-param tindex_delta=0" ;;
        c5) args="--config5-only --no-pmc --no-cpu" ;;
    esac
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$leg -o $leg -- python3 $R/bench.py $args > $O/$leg.json 2> $O/$leg.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "leg $leg failed rc=$rc"; tail -20 $O/$leg.err; exit 1; fi
    echo "== $leg"; tail -c 3000 $O/$leg.json; echo
    head -12 $O/$leg/${leg}_kernel_stats.csv | cut -d, -f1-4
done
