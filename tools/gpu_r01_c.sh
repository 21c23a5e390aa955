cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 700 python -m pytest tests -q -m gpu --maxfail=30 > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --config c3 --steps 5 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
rc=$?; echo "bench c3 rc=$rc"; cat gpurun_out/bench_c3.json; tail -3 gpurun_out/bench_c3.err
exit $rc
