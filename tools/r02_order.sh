# scan_order A/B: C5 with/without (plus contain_skip), C3 regression check
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r02ord}
mkdir -p $O
for v in "" "--opt scan_order=1" "--opt contain_skip=0"; do
  tag=$(echo "$v" | tr -d ' -=' | tr -c 'a-z0-9\n' '_')
  timeout -k 10 400 python -u bench.py --config c5 --steps 2 --no-cpu-baseline --no-ingest $v > $O/c5_$tag.json 2> $O/c5_$tag.err
  rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc $v"; tail -5 $O/c5_$tag.err; exit $rc; }
  python3 -c "import json;d=json.load(open('$O/c5_$tag.json'));print('$v', 'ms', round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['device_ms'].items() if k in ('index_ms','contained_ms','probe_ms')}, {k:v for k,v in d['counters'].items() if k.startswith('c_') or k=='verified' or k=='runs'}, d['parity']['super']['sum'], d['parity']['rows']['sum'])"
done
timeout -k 10 400 python -u bench.py --steps 5 --no-cpu-baseline --no-ingest > $O/c3.json 2> $O/c3.err
rc=$?; python3 -c "import json;d=json.load(open('$O/c3.json'));print('c3 ms', round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['device_ms'].items()}, d['parity']['digest_ok'])"; exit $rc
