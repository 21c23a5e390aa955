cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -q -m gpu -x -k "fixture or random" > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --config c3 --steps 5 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
rc=$?; echo "bench c3 rc=$rc"; cat gpurun_out/bench_c3.json; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/gpu_pmc.sh c2 r01 > gpurun_out/pmc.log 2>&1
rc=$?; tail -5 gpurun_out/pmc.log; exit $rc
