cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r02m}
mkdir -p $O
MG_VARIANTS="${2}" timeout -k 10 400 python -u tools/variant_sweep.py > $O/sweep.log 2>&1; rc=$?
grep opts $O/sweep.log; exit $rc
