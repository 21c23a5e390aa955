cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
echo "host: $(nproc) cpus"; rocm-smi --showproductname 2>&1 | head -8
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -m pytest tests -q -m gpu --maxfail=30 > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config c2 --steps 5 --no-cpu-baseline > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_c2.json; tail -5 gpurun_out/bench_c2.err
exit $rc
