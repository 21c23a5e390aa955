#!/bin/bash
# A/B of alternative library builds (metagenomics_amd/lib/variants/*.so) against
# the default build, alternating in separate processes on one box.
#   usage: tools/ab_libs.sh TAG
cd $GRAFT_REPO_ROOT
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export MG_VARIANTS=${MG_VARIANTS:-'[{}, {}]'}
for rep in 1 2; do
  for L in default metagenomics_amd/lib/variants/*.so; do
    if [ "$L" = default ]; then unset MG_LIB; else export MG_LIB=$PWD/$L; fi
    timeout -k 10 300 python -u tools/variant_sweep.py > $OUT/ab_$(basename $L)_$rep.log 2>&1
    rc=$?; echo "$L rep $rep rc=$rc"; grep opts $OUT/ab_$(basename $L)_$rep.log; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
