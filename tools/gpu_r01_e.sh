cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -q -m gpu --maxfail=10 -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python tools/phase_sweep.py 10000000 > gpurun_out/phase_sweep.log 2>&1
rc=$?; grep -v "^{" gpurun_out/phase_sweep.log; exit $rc
