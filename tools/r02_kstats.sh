# kernel-trace stats of the C3 bench under engine options (MG_BENCH_OPTS json)
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r02k}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o kt -- python3 bench.py --steps 3 --no-cpu-baseline --no-ingest ${2} > $O/prof_bench.json 2> $O/prof_bench.err
rc=$?; python3 -c "import json;d=json.load(open('$O/prof_bench.json'));print('ms/step',round(d['ms_per_step'],3),{k:round(v,3) for k,v in d['device_ms'].items()})"
cut -d, -f1-4 $O/prof/kt_kernel_stats.csv | sed 's/(anonymous namespace):://g' | cut -c1-150 | head -16; exit $rc
