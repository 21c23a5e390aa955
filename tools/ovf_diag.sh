#!/bin/bash
# TEMP: overflow / bin-size distribution of the exchange mode's cell build (MG_DEBUG_OVF)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ovf
MG_DEBUG_OVF=1 timeout -k 10 300 python -u bench.py --config ${1:-c5s} --sim-world 8 --multi exchange --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --opt layout_scratch=0 > gpurun_out/ovf/run.json 2> gpurun_out/ovf/run.err
rc=$?
grep "\[ovf\]" gpurun_out/ovf/run.err | head -40
exit $rc
