# probe_share_xcd: option tests, C3 A/B (alternating, one process)
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r02sx}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "containment_options" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -ne 0 ] && exit $rc
export MG_VARIANTS='[{}, {"probe_share_xcd": 1}, {}, {"probe_share_xcd": 1}, {}, {"probe_share_xcd": 1}, {}, {"probe_share_xcd": 1}]'
timeout -k 10 500 python -u tools/variant_sweep.py > $O/sweep.log 2>&1; rc=$?; grep opts $O/sweep.log; exit $rc
