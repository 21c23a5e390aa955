cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r02c
export MG_VARIANTS='[{}, {"scan_reg":0}, {"overlap_scan":0}, {"overlap_scan":0,"scan_reg":0}, {}, {"scan_reg":0}, {"overlap_scan":0}, {"overlap_scan":0,"scan_reg":0}]'
timeout -k 10 400 python -u tools/variant_sweep.py > gpurun_out/r02c/sweep.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02c/prof -o kt -- python3 bench.py --steps 5 --no-cpu-baseline --no-ingest > gpurun_out/r02c/prof_bench.json 2> gpurun_out/r02c/prof_bench.err
rc=$?; cat gpurun_out/r02c/sweep.log | grep opts; head -12 gpurun_out/r02c/prof/kt_kernel_stats.csv | cut -c1-160; exit $rc
