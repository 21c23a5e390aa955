# reg_cas: tests, C3 A/B (one process, alternating), C5 A/B
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r02rc}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "reg_cas or containment_options" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
export MG_VARIANTS='[{}, {"reg_cas": 1}, {}, {"reg_cas": 1}, {}, {"reg_cas": 1}]'
timeout -k 10 500 python -u tools/variant_sweep.py > $O/sweep.log 2>&1; rc=$?; grep opts $O/sweep.log; [ $rc -ne 0 ] && exit $rc
for v in "" "--opt reg_cas=1"; do
  tag=$(echo "$v" | sed 's/[^a-z0-9]/_/g')
  timeout -k 10 400 python -u bench.py --config c5 --steps 2 --no-cpu-baseline --no-ingest $v > $O/c5_$tag.json 2> $O/c5_$tag.err
  rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc $v"; tail -5 $O/c5_$tag.err; exit $rc; }
  python3 -c "import json;d=json.load(open('$O/c5_$tag.json'));print('c5 $v', 'ms', round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['device_ms'].items() if k in ('index_ms','scan_ms','contained_ms','probe_ms')}, d['parity']['super']['sum'], d['parity']['rows']['sum'])"
done
