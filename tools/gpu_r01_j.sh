# kernel-trace stats of the C3 bench + PMC counter passes (each its own run)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_j
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_j -o kt -- python3 bench.py --config c3 --steps 5 --no-cpu-baseline > gpurun_out/prof_j/bench.json 2> gpurun_out/prof_j/bench.err
rc=$?; echo "stats rc=$rc"; cat gpurun_out/prof_j/bench.json; if [ $rc -ne 0 ]; then tail -20 gpurun_out/prof_j/bench.err; exit $rc; fi
bash tools/gpu_pmc.sh c3 j
