cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 700 python -m pytest tests -q -m gpu -x > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python tools/phase_sweep.py 10000000 > gpurun_out/phase_sweep.log 2>&1
rc=$?; grep -v "^{" gpurun_out/phase_sweep.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --config c3 --steps 5 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
rc=$?; echo "bench c3 rc=$rc"; cat gpurun_out/bench_c3.json; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 tools/micro/gather_bench 600 200000000 > gpurun_out/gather.json 2>&1
rc=$?; echo "gather rc=$rc"; cat gpurun_out/gather.json; exit $rc
