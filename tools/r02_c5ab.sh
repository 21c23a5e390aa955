# C5-shaped A/B: join vs cell path (bench.py --config c5s / c5)
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r02l}
CFG=${2:-c5s}
mkdir -p $O
for opt in "join=1" "join=0"; do
  timeout -k 10 400 python -u bench.py --config $CFG --steps 3 --no-cpu-baseline --no-ingest --opt $opt > $O/bench_${CFG}_$opt.json 2> $O/bench_${CFG}_$opt.err || exit 1
  python3 -c "import json;d=json.load(open('$O/bench_${CFG}_$opt.json'));print('$opt', 'ms/step',round(d['ms_per_step'],3),{k:round(v,3) for k,v in d['device_ms'].items()}, d['parity']['digest_ok'])"
done
