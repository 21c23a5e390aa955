# round-6 exchange iteration: exchange parity tests, then per-rank kernel tables (C3, P = 2 and 8)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && T=${1:-r06x} && mkdir -p gpurun_out/$T
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py tests/test_xchg_host.py -x -q -m gpu -k "exchange or allocation or fixtures_p3 or worlds or route or rerun" --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/$T/tests.log; [ $rc -ne 0 ] && { grep -E "FAIL|Error" gpurun_out/$T/tests.log | head -20; exit $rc; }
SIMC=${SIMC:-c3} SIMP=${SIMP:-"2 8"} bash tools/gpu_run.sh $T profsimP || exit 1
[ -n "$ABOPTS" ] && SIMC=${SIMC:-c3} SIMP=${ABP:-8} SIMOPTS="$ABOPTS" bash tools/gpu_run.sh ${T}_ab profsimP
exit 0
