# GPU suite, then C3 and C5 benches (stats pass prints the work counters)
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r02ch}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
for cfg in c3 c5; do
  timeout -k 10 400 python -u bench.py --config $cfg --steps 3 --no-cpu-baseline --no-ingest > $O/$cfg.json 2> $O/$cfg.err
  rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc $cfg"; tail -5 $O/$cfg.err; exit $rc; }
  python3 -c "import json;d=json.load(open('$O/$cfg.json'));print('$cfg', 'ms', round(d['ms_per_step'],3), {k:round(v,2) for k,v in d['device_ms'].items() if k in ('index_ms','contained_ms','probe_ms')}, {k:v for k,v in d['counters'].items()}, d['parity'].get('digest_ok'), d['parity']['super']['sum'], d['parity']['rows']['sum'])"
done
