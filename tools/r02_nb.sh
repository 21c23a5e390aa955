# C3 step under directory sizes (nb_log2 23 / auto 24 / 25), alternating, one process
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r02nb}
mkdir -p $O
export MG_VARIANTS='[{}, {"nb_log2": 23}, {"nb_log2": 25}, {}, {"nb_log2": 23}, {"nb_log2": 25}]'
timeout -k 10 500 python -u tools/variant_sweep.py > $O/sweep.log 2>&1; rc=$?; cat $O/sweep.log | grep opts; exit $rc
