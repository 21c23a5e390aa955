cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 700 python -m pytest tests -q -m gpu --maxfail=30 > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/gpu_tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --config c3 --steps 5 --no-cpu-baseline > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err
rc=$?; echo "bench c3 rc=$rc"; cat gpurun_out/bench_c3.json
if [ $rc -ne 0 ]; then exit $rc; fi
for mode in buckets reads; do
timeout -k 10 300 python bench.py --config c3 --steps 3 --no-cpu-baseline --sim-world 8 --shard $mode > gpurun_out/bench_c3_sim8_$mode.json 2>/dev/null
rc=$?; echo "sim8 $mode rc=$rc"; python -c "import json;d=json.load(open('gpurun_out/bench_c3_sim8_$mode.json'));print(d['ms_per_step'], d['device_ms'])"
if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r01 --output-format csv -- python bench.py --config c3 --steps 3 --warmup 0 --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; find gpurun_out/prof -name "*stats*" | head; 
exit $rc
