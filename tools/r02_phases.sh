# probe phase split on the default (bucket-sorted) path and the unsorted path
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02d
timeout -k 10 400 python -u tools/phase_sweep.py > gpurun_out/r02d/phases_sorted.log 2>&1 && \
MG_SORT_RUNS=0 timeout -k 10 400 python -u tools/phase_sweep.py > gpurun_out/r02d/phases_unsorted.log 2>&1
rc=$?; grep phase gpurun_out/r02d/phases_*.log; exit $rc
