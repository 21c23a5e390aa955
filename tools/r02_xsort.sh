# exchange mode: full bucket sort of the runs vs top-8-bit sort (routing needs only the owner bits), simulated ranks
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r02xs}
mkdir -p $O
for P in 8 2; do
  for v in "" "--opt sort_bits=8" "--opt sort_bits=12"; do
    tag=sim${P}$(echo "$v" | sed 's/[^a-z0-9]/_/g')
    timeout -k 10 300 python -u bench.py --sim-world $P --multi exchange --steps 3 --no-cpu-baseline --no-ingest $v > $O/$tag.json 2> $O/$tag.err
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc $P $v"; tail -5 $O/$tag.err; exit $rc; }
    python3 -c "import json;d=json.load(open('$O/$tag.json'));print('P=$P $v ms/step',round(d['ms_per_step'],3),'digest_ok',d['parity'].get('digest_ok'),{k:round(v,2) for k,v in d['device_ms'].items() if k in ('scan_ms','sort_ms','probe_ms','index_ms')})"
  done
done
