# partner prefetch: option-matrix + fixture tests with it, C3 A/B (alternating, one process), C5 A/B
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r02pf}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
export MG_VARIANTS='[{}, {"probe_prefetch": 1}, {}, {"probe_prefetch": 1}, {}, {"probe_prefetch": 1}]'
timeout -k 10 500 python -u tools/variant_sweep.py > $O/sweep.log 2>&1; rc=$?; grep opts $O/sweep.log; [ $rc -ne 0 ] && exit $rc
for v in "" "--opt probe_prefetch=1"; do
  tag=$(echo "$v" | sed 's/[^a-z0-9]/_/g')
  timeout -k 10 400 python -u bench.py --config c5 --steps 2 --no-cpu-baseline --no-ingest $v > $O/c5_$tag.json 2> $O/c5_$tag.err
  rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc $v"; tail -5 $O/c5_$tag.err; exit $rc; }
  python3 -c "import json;d=json.load(open('$O/c5_$tag.json'));print('c5 $v', 'ms', round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['device_ms'].items() if k in ('index_ms','contained_ms','probe_ms')}, d['parity']['super']['sum'], d['parity']['rows']['sum'])"
done
