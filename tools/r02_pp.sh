# pp scan: parity subset, then C3 A/B in one process
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-pp}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k "scan_pp" --timeout 300 --timeout-method thread > $O/pp_tests.log 2>&1
rc=$?; echo "pp tests rc=$rc"; grep -E "passed|failed|Error|assert" $O/pp_tests.log | tail -15; [ $rc -ne 0 ] && exit $rc
export MG_VARIANTS='[{}, {"scan_pp":1}, {}, {"scan_pp":1}, {"scan_pp":1,"sort_runs":0}, {"sort_runs":0}]'
timeout -k 10 400 python -u tools/variant_sweep.py > $O/sweep.log 2>&1; rc=$?; grep opts $O/sweep.log; exit $rc
