# C3 probe region mapping: scan-wave regions as dealt (default) vs XCD-contiguous (xcd_plain), alternating, one process
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r02xcd}
mkdir -p $O
export MG_VARIANTS='[{}, {"xcd_plain": 1}, {}, {"xcd_plain": 1}, {}, {"xcd_plain": 1}]'
timeout -k 10 500 python -u tools/variant_sweep.py > $O/sweep.log 2>&1; rc=$?; grep opts $O/sweep.log; exit $rc
