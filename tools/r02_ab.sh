# full GPU suite (optional), then a C3 variant sweep (MG_VARIANTS) in one process
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-ab}
mkdir -p $O
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 500 python -u tools/variant_sweep.py > $O/sweep.log 2>&1; rc=$?; grep opts $O/sweep.log; exit $rc
