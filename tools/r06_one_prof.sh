export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r06
mkdir -p $O
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/one_prof -o one -- python3 $GRAFT_REPO_ROOT/tools/r05_one.py > $O/one_prof.txt 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/one_prof_sparse -o one -- python3 $GRAFT_REPO_ROOT/tools/r05_one.py 10000000 sparse > $O/one_prof_sparse.txt 2>&1 || exit 1
grep "R=1" $O/one_prof.txt $O/one_prof_sparse.txt
