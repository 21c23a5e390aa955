# rocprofv3 counter passes (each its own run; --kernel-trace only, no sys/runtime trace)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
CFG=${1:-c2}
TAG=${2:-r01}
mkdir -p gpurun_out/pmc_$TAG
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SMEM" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  echo "pass $i: $set"
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/pmc_$TAG/p$i -o p$i -- python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_$TAG/p$i.log 2>&1
  rc=$?; echo "rc=$rc"; if [ $rc -ne 0 ]; then tail -20 gpurun_out/pmc_$TAG/p$i.log; break; fi
done
python3 tools/pmc_summary.py gpurun_out/pmc_$TAG/summary.json gpurun_out/pmc_$TAG/p* > /dev/null
exit $rc
