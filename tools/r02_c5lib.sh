# C5 A/B of library builds (metagenomics_amd/lib/variants/*.so vs default), alternating processes
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r02c5lib}
mkdir -p $O
for rep in 1 2; do
  for L in default metagenomics_amd/lib/variants/*.so; do
    if [ "$L" = default ]; then unset MG_LIB; else export MG_LIB=$PWD/$L; fi
    tag=$(basename $L .so)_$rep
    timeout -k 10 400 python -u bench.py --config c5 --steps 2 --no-cpu-baseline --no-ingest > $O/c5_$tag.json 2> $O/c5_$tag.err
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc $L"; tail -5 $O/c5_$tag.err; exit $rc; }
    python3 -c "import json;d=json.load(open('$O/c5_$tag.json'));print('c5 $tag', 'ms', round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['device_ms'].items() if k in ('index_ms','scan_ms','contained_ms','probe_ms')}, d['parity']['super']['sum'], d['parity']['rows']['sum'])"
  done
done
