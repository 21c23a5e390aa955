cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v1
export MG_VARIANTS='[{}, {"probe_region":128,"xcd_map":1}, {"probe_region":256,"xcd_map":1}, {"probe_region":64,"xcd_map":1}, {"probe_region":128,"xcd_map":0}, {"sort_bits":16,"probe_region":128,"xcd_map":1}, {"sort_bits":12,"probe_region":128,"xcd_map":1}, {"sort_bits":8,"probe_region":128,"xcd_map":1}, {}, {"probe_region":128,"xcd_map":1}]'
timeout -k 10 500 python -u tools/variant_sweep.py > gpurun_out/v1/sweep.log 2>&1; rc=$?; cat gpurun_out/v1/sweep.log | grep opts; exit $rc
