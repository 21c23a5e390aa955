cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02opt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -k "containment_options" --timeout 300 --timeout-method thread > gpurun_out/r02opt/opt_tests.log 2>&1
rc=$?; echo "opt tests rc=$rc"; grep -E "PASS|FAIL|Error" gpurun_out/r02opt/opt_tests.log | tail -8; [ $rc -ne 0 ] && exit $rc
bash tools/r02_order.sh r02ord
