# ping-pong cell tables: GPU suite, then C3 bench wall (default cell_pp=1 vs 0), alternating processes
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r02pp}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for v in "" "--opt cell_pp=0"; do
    tag=$(echo "$v" | sed 's/[^a-z0-9]/_/g')_$rep
    timeout -k 10 400 python -u bench.py --steps 10 --no-cpu-baseline --no-ingest $v > $O/c3_$tag.json 2> $O/c3_$tag.err
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc $v"; tail -5 $O/c3_$tag.err; exit $rc; }
    python3 -c "import json;d=json.load(open('$O/c3_$tag.json'));print('c3 $v', 'wall ms', round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['device_ms'].items() if k in ('index_ms','scan_ms','probe_ms','total_ms')}, d['parity']['digest_ok'])"
  done
done
