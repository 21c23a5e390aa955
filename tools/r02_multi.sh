# multi-GPU readiness on one box: one-rank RCCL exchange step (torchrun), simulated exchange ranks P = 2/4/8,
# then a C5 A/B of the register scan as the index build (reg_index)
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh ${1:-r02mg} xchg1 sim || exit $?
O=gpurun_out/${1:-r02mg}
for v in "" "--opt reg_index=1"; do
  tag=$(echo "$v" | sed 's/[^a-z0-9]/_/g')
  timeout -k 10 400 python -u bench.py --config c5 --steps 2 --no-cpu-baseline --no-ingest $v > $O/c5_$tag.json 2> $O/c5_$tag.err
  rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc $v"; tail -5 $O/c5_$tag.err; exit $rc; }
  python3 -c "import json;d=json.load(open('$O/c5_$tag.json'));print('c5 $v', 'ms', round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['device_ms'].items() if k in ('index_ms','contained_ms','probe_ms')}, d['parity']['super']['sum'], d['parity']['rows']['sum'])"
done
