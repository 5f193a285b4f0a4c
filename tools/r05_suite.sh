#!/bin/bash
# Round 5: the whole GPU suite (with the slowest durations), then optional A/B legs and a kernel trace.
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r05s
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider --durations=30 > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head -20; exit $rc; }
if [ -n "$AB" ]; then bash tools/r05_libab.sh $AB || exit 1; fi
if [ -n "$PROF" ]; then bash tools/r05_metric.sh "" || exit 1; fi
