cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02lr
timeout -k 10 600 python -u -m pytest tests/test_long_reads.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r02lr/long.log 2>&1
rc=$?; echo "long rc=$rc"; grep -E "PASS|FAIL|Error|error" gpurun_out/r02lr/long.log | tail -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r02lr/gpu_tests.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -15 gpurun_out/r02lr/gpu_tests.log; exit $rc
