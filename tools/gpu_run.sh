#!/bin/bash
# One GPU-box session: parity tests, C3 bench (with CPU baseline), rocprofv3
# kernel-trace stats of the same bench command, and FETCH_SIZE / WRITE_SIZE PMC
# passes (each its own run, --kernel-trace only).  Every GPU step has its own
# time limit; the first failure ends the script.
#   usage: tools/gpu_run.sh TAG [tests|bench|prof|pmc ...]   (default: all)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-run}; shift
STEPS=${@:-tests bench prof pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for s in $STEPS; do
  case $s in
  tests)
    timeout -k 10 1150 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
    rc=$?; echo "tests rc=$rc"; tail -3 $OUT/gpu_tests.log ;;
  smoke)
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
    rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log ;;
  bench)
    timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
    rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json ;;
  sim)
    for P in 2 4 8; do
      timeout -k 10 300 python -u bench.py --sim-world $P --multi exchange --steps 3 --no-cpu-baseline --no-ingest > $OUT/bench_sim$P.json 2> $OUT/bench_sim$P.err
      rc=$?; echo "bench sim $P rc=$rc"; python3 -c "import json;d=json.load(open('$OUT/bench_sim$P.json'));print('ms/step',round(d['ms_per_step'],3),'digest_ok',d['parity'].get('digest_ok'),'reruns',d.get('exchange_reruns'),d.get('phase_wall_ms'))"; [ $rc -ne 0 ] && break
    done ;;
  simrep)
    for P in 2 4 8; do
      timeout -k 10 600 python -u bench.py --config ${SIMREP_CONFIG:-c3} --sim-world $P --multi replicated --steps 3 --no-cpu-baseline --no-ingest $SIMOPTS > $OUT/bench_simrep${P}_${SIMREP_CONFIG:-c3}.json 2> $OUT/bench_simrep$P.err
      rc=$?; echo "bench sim replicated $P rc=$rc"; python3 -c "import json;d=json.load(open('$OUT/bench_simrep${P}_${SIMREP_CONFIG:-c3}.json'));print(round(d['ms_per_step'],3), d['value'], d['undirected_edges'], d['parity'].get('digest_ok'), [round(x,3) for x in d.get('sim_rank_ms')], {k:round(v,3) for k,v in d['device_ms'].items()})"; [ $rc -ne 0 ] && break
    done ;;
  simbkt)
    for P in ${SIMP:-2 4 8}; do
      timeout -k 10 600 python -u bench.py --config ${SIMREP_CONFIG:-c3} --sim-world $P --multi bucket --steps 3 --no-cpu-baseline --no-ingest $SIMOPTS > $OUT/bench_simbkt${P}_${SIMREP_CONFIG:-c3}.json 2> $OUT/bench_simbkt$P.err
      rc=$?; echo "bench sim bucket $P rc=$rc"; python3 -c "import json;d=json.load(open('$OUT/bench_simbkt${P}_${SIMREP_CONFIG:-c3}.json'));print(round(d['ms_per_step'],3), d['value'], d['undirected_edges'], d['parity'].get('digest_ok'), [round(x,3) for x in d.get('sim_rank_ms')], {k:round(v,3) for k,v in d['device_ms'].items()})"; [ $rc -ne 0 ] && break
    done ;;
  xchg1)
    timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --exchange --steps 5 --no-cpu-baseline --no-ingest > $OUT/bench_xchg1.json 2> $OUT/bench_xchg1.err
    rc=$?; echo "bench exchange(RCCL, 1 rank) rc=$rc"; python3 -c "import json;d=json.load(open('$OUT/bench_xchg1.json'));print('ms/step',round(d['ms_per_step'],3),'edges',d['undirected_edges'],'digest_ok',d['parity'].get('digest_ok'),'reruns',d.get('exchange_reruns'),{k:round(v,3) for k,v in d['device_ms'].items()},d.get('phase_wall_ms'))" ;;
  profxchg1)
    export MASTER_ADDR=127.0.0.1 MASTER_PORT=29513 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profxchg1 -o kt -- python3 bench.py --exchange --steps 5 --no-cpu-baseline --no-ingest > $OUT/profxchg1_bench.json 2> $OUT/profxchg1_bench.err
    rc=$?; unset MASTER_ADDR MASTER_PORT RANK WORLD_SIZE LOCAL_RANK; echo "profxchg1 rc=$rc"; cat $OUT/profxchg1_bench.json; head -24 $OUT/profxchg1/kt_kernel_stats.csv | cut -c1-160 ;;
  newtests)
    timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_long_reads.py -x -v -m gpu -k "${KT:-exchange or live_index or falls_back}" --timeout 300 --timeout-method thread > $OUT/new_tests.log 2>&1
    rc=$?; echo "new tests rc=$rc"; grep -E "PASS|FAIL|Error" $OUT/new_tests.log | tail -40 ;;
  xdigest)
    timeout -k 10 1100 python -u -m pytest tests/test_scale_digest.py -x -v -m gpu -k "exchange_scale" --timeout 1000 --timeout-method thread > $OUT/xdigest_tests.log 2>&1
    rc=$?; echo "exchange digest tests rc=$rc"; grep -E "PASS|FAIL|SKIP|Error" $OUT/xdigest_tests.log | tail -12 ;;
  xchgtests)
    timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v -m gpu -k exchange --timeout 300 --timeout-method thread > $OUT/xchg_tests.log 2>&1
    rc=$?; echo "exchange tests rc=$rc"; grep -E "PASS|FAIL|Error" $OUT/xchg_tests.log | tail -20 ;;
  digest)
    timeout -k 10 1100 python -u -m pytest tests/test_scale_digest.py -x -v -m gpu --timeout 900 --timeout-method thread > $OUT/digest_tests.log 2>&1
    rc=$?; echo "digest tests rc=$rc"; grep -E "PASS|FAIL|SKIP|Error" $OUT/digest_tests.log | tail -12 ;;
  parity)
    timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_hashtable_api.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/parity_tests.log 2>&1
    rc=$?; echo "parity tests rc=$rc"; tail -3 $OUT/parity_tests.log ;;
  c3digest)
    timeout -k 10 900 python -u -m pytest tests/test_scale_digest.py -x -v -m gpu -k "c3 or c5s" --timeout 900 --timeout-method thread > $OUT/c3digest_tests.log 2>&1
    rc=$?; echo "c3/c5s digest tests rc=$rc"; grep -E "PASS|FAIL|SKIP|Error" $OUT/c3digest_tests.log | tail -12 ;;
  clixchg)
    timeout -k 10 1000 python -u -m pytest tests/test_scale_digest.py -x -v -m gpu -k cli_exchange --timeout 900 --timeout-method thread > $OUT/clixchg_tests.log 2>&1
    rc=$?; echo "cli exchange tests rc=$rc"; grep -E "PASS|FAIL|SKIP|Error|assert" $OUT/clixchg_tests.log | tail -12 ;;
  profsim8)
    # per-rank kernel tables of the exchange mode at P=8 (simulated ranks, one rank's call at a
    # time: MG_SIM_SERIAL), C3 then C5
    for C in c3 c5; do
      MG_SIM_SERIAL=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profsim8_$C -o kt -- python3 bench.py --config $C --sim-world 8 --multi exchange --steps 2 --no-cpu-baseline --no-ingest --opt layout_scratch=0 $SIMOPTS > $OUT/profsim8_${C}_bench.json 2> $OUT/profsim8_${C}_bench.err
      rc=$?; echo "profsim8 $C rc=$rc"; [ $rc -ne 0 ] && break
      python3 tools/rank_table.py $OUT/profsim8_$C/kt_kernel_stats.csv 8 4 "$C exchange-sim" | tee $OUT/profsim8_${C}_ranks.md | tail -14
    done ;;
  simab)
    # wall of the simulated exchange step (serial ranks) for option A/B pairs: MG_AB="opt=v ..." vs default
    for C in ${SIMAB_CONFIGS:-c3 c5}; do
      for rep in 1 2; do
        for V in "" "$MG_AB"; do
          o=""; for kv in $V; do o="$o --opt $kv"; done
          MG_SIM_SERIAL=1 timeout -k 10 400 python -u bench.py --config $C --sim-world 8 --multi exchange --steps 3 --no-cpu-baseline --no-ingest --opt layout_scratch=0 $o > $OUT/simab.json 2> $OUT/simab.err
          rc=$?; [ $rc -ne 0 ] && break 3
          python3 -c "import json;d=json.load(open('$OUT/simab.json'));print('$C','[$V]','ms/step',round(d['ms_per_step'],3),'digest_ok',d['parity'].get('digest_ok'),{k:round(v,2) for k,v in (d.get('phase_wall_ms') or {}).items()})" | tee -a $OUT/simab.log
        done
      done
    done ;;
  fusedab)
    # fused-path option A/B pairs (alternating processes, one box): MG_AB="opt=v ..." vs default,
    # configs in FUSEDAB_CONFIGS (default c5)
    for C in ${FUSEDAB_CONFIGS:-c5}; do
      for rep in 1 2; do
        for V in "" "$MG_AB"; do
          o=""; for kv in $V; do o="$o --opt $kv"; done
          timeout -k 10 400 python -u bench.py --config $C --steps 5 --no-cpu-baseline --no-ingest --no-one-shot --no-d2h $o > $OUT/fusedab.json 2> $OUT/fusedab.err
          rc=$?; [ $rc -ne 0 ] && break 3
          python3 -c "import json;d=json.load(open('$OUT/fusedab.json'));print('$C','[$V]','ms/step',round(d['ms_per_step'],3),'digest_ok',d['parity'].get('digest_ok'),{k:round(v,3) for k,v in d['device_ms'].items() if v})" | tee -a $OUT/fusedab.log
        done
      done
    done ;;
  optsweep)
    # one fused bench per option set: OPTSETS="a=1 b=2;c=3;..." ("" = default), config SWEEP_CONFIG (c5)
    IFS=';' read -ra sets <<< "${OPTSETS}"
    for V in "" "${sets[@]}"; do
      o=""; for kv in $V; do o="$o --opt $kv"; done
      timeout -k 10 400 python -u bench.py --config ${SWEEP_CONFIG:-c5} --steps 3 --no-cpu-baseline --no-ingest --no-one-shot --no-d2h $o > $OUT/optsweep.json 2> $OUT/optsweep.err
      rc=$?; [ $rc -ne 0 ] && break
      python3 -c "import json;d=json.load(open('$OUT/optsweep.json'));print('${SWEEP_CONFIG:-c5}','[$V]','ms/step',round(d['ms_per_step'],3),'digest_ok',d['parity'].get('digest_ok'),{k:round(v,3) for k,v in d['device_ms'].items() if v},{k:v for k,v in d['counters'].items() if v})" | tee -a $OUT/optsweep.log
    done ;;
  libab)
    # variant libraries (metagenomics_amd/lib/variants/NAME.so, LIBS="a b") against the default
    # build, alternating processes, config LIBAB_CONFIG (c5)
    for rep in 1 2; do
      for L in default $LIBS; do
        if [ "$L" = default ]; then lib=""; else lib=$PWD/metagenomics_amd/lib/variants/$L.so; fi
        MG_LIB=$lib timeout -k 10 400 python -u bench.py --config ${LIBAB_CONFIG:-c5} --steps 5 --no-cpu-baseline --no-ingest --no-one-shot --no-d2h > $OUT/libab.json 2> $OUT/libab.err
        rc=$?; [ $rc -ne 0 ] && break 2
        python3 -c "import json;d=json.load(open('$OUT/libab.json'));print('${LIBAB_CONFIG:-c5}','$L','ms/step',round(d['ms_per_step'],3),'digest_ok',d['parity'].get('digest_ok'),{k:round(v,3) for k,v in d['device_ms'].items() if v})" | tee -a $OUT/libab.log
      done
    done ;;
  a2a)
    timeout -k 10 300 python -u tools/a2a_probe.py > $OUT/a2a_probe.log 2>&1
    rc=$?; echo "a2a_probe rc=$rc"; grep MB $OUT/a2a_probe.log ;;
  benchq)
    timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/benchq.json 2> $OUT/benchq.err
    rc=$?; echo "benchq rc=$rc"; python3 -c "import json;d=json.load(open('$OUT/benchq.json'));print('ms/step',round(d['ms_per_step'],3),'edges',d['undirected_edges'],{k:round(v,3) for k,v in d['device_ms'].items()})" ;;
  replay)
    timeout -k 10 600 python -u bench.py --replay --no-cpu-baseline --no-ingest --steps 2 > $OUT/bench_replay.json 2> $OUT/bench_replay.err
    rc=$?; echo "bench replay rc=$rc"; python3 -c "import json;d=json.load(open('$OUT/bench_replay.json'));print(d.get('graph_replay'))" ;;
  parse)
    timeout -k 10 900 python -u tools/parse_bench.py > $OUT/parse_bench.json 2> $OUT/parse_bench.err
    rc=$?; echo "parse rc=$rc"; tail -12 $OUT/parse_bench.err; cat $OUT/parse_bench.json ;;
  sweep)
    timeout -k 10 600 python -u tools/variant_sweep.py > $OUT/sweep_${MG_SWEEP_CONFIG:-c3}.log 2>&1
    rc=$?; echo "sweep rc=$rc"; grep opts $OUT/sweep_${MG_SWEEP_CONFIG:-c3}.log ;;
  variants)
    timeout -k 10 400 python -u tools/variant_sweep.py > $OUT/variant_sweep.log 2>&1
    rc=$?; echo "variants rc=$rc"; grep opts $OUT/variant_sweep.log ;;
  phases)
    timeout -k 10 400 python -u tools/phase_sweep.py > $OUT/phase_sweep.log 2>&1
    rc=$?; echo "phases rc=$rc"; grep phase $OUT/phase_sweep.log ;;
  benchc2)
    timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err
    rc=$?; echo "bench c2 rc=$rc"; cat $OUT/bench_c2.json ;;
  benchc5)
    timeout -k 10 600 python -u bench.py --config c5 --no-ingest > $OUT/bench_c5.json 2> $OUT/bench_c5.err
    rc=$?; echo "bench c5 rc=$rc"; cat $OUT/bench_c5.json ;;
  benchc5s)
    timeout -k 10 300 python -u bench.py --config c5s --no-cpu-baseline --no-ingest > $OUT/bench_c5s.json 2> $OUT/bench_c5s.err
    rc=$?; echo "bench c5s rc=$rc"; cat $OUT/bench_c5s.json ;;
  prof)
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o kt -- python3 bench.py --steps 5 --no-cpu-baseline --no-ingest --no-one-shot > $OUT/prof_bench.json 2> $OUT/prof_bench.err
    rc=$?; echo "prof rc=$rc"; cat $OUT/prof_bench.json; head -8 $OUT/prof/kt_kernel_stats.csv | cut -c1-200 ;;
  profsim)
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profsim -o kt -- python3 bench.py --sim-world 4 --multi exchange --steps 2 --no-cpu-baseline > $OUT/profsim_bench.json 2> $OUT/profsim_bench.err
    rc=$?; echo "profsim rc=$rc"; cat $OUT/profsim_bench.json; cat $OUT/profsim/kt_kernel_stats.csv ;;
  pmclist)
    timeout -k 10 120 rocprofv3 -L > $OUT/counters_all.txt 2>&1
    rc=$?; echo "pmclist rc=$rc"; grep -oE '\b(TA|TD|TCP|TCC)_[A-Z0-9_]+' $OUT/counters_all.txt | sort -u > $OUT/counters_mem.txt; wc -l $OUT/counters_mem.txt ;;
  pmcset)
    # one pass per $PMCSETS entry (';'-separated counter sets) over a 1-step C3 bench
    i=0; IFS=';' read -ra SETS <<< "$PMCSETS"
    for set in "${SETS[@]}"; do
      i=$((i+1))
      timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/pmcset_$i -o p -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --no-one-shot > $OUT/pmcset_$i.log 2>&1
      rc=$?; echo "pmcset $i rc=$rc"; [ $rc -ne 0 ] && break
    done
    [ $rc -eq 0 ] && python3 tools/pmc_summary.py $OUT/pmcset_summary.json $OUT/pmcset_* > /dev/null ;;
  pmcsq)
    i=0
    for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
               "SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
      i=$((i+1))
      timeout -s KILL 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/pmcsq_$i -o p -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --no-one-shot > $OUT/pmcsq_$i.log 2>&1
      rc=$?; echo "pmcsq $i rc=$rc"; [ $rc -ne 0 ] && break
    done
    [ $rc -eq 0 ] && python3 tools/pmc_summary.py $OUT/pmcsq_summary.json $OUT/pmcsq_* > /dev/null ;;
  pmc)
    for set in "FETCH_SIZE" "WRITE_SIZE"; do
      timeout -s KILL 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/pmc_$set -o p -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --no-one-shot > $OUT/pmc_$set.log 2>&1
      rc=$?; echo "pmc $set rc=$rc"; [ $rc -ne 0 ] && break
    done
    [ $rc -eq 0 ] && python3 tools/pmc_summary.py $OUT/pmc_summary.json $OUT/pmc_* > /dev/null ;;
  pmc5)
    for set in "FETCH_SIZE" "WRITE_SIZE"; do
      timeout -s KILL 400 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/pmc5_$set -o p -- python3 bench.py --config c5 --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --no-one-shot > $OUT/pmc5_$set.log 2>&1
      rc=$?; echo "pmc5 $set rc=$rc"; [ $rc -ne 0 ] && break
    done
    [ $rc -eq 0 ] && python3 tools/pmc_summary.py $OUT/pmc5_summary.json $OUT/pmc5_* > /dev/null ;;
  prof5)
    timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof5 -o kt -- python3 bench.py --config c5 --steps 2 --no-cpu-baseline --no-ingest --no-one-shot > $OUT/prof5_bench.json 2> $OUT/prof5_bench.err
    rc=$?; echo "prof5 rc=$rc"; head -10 $OUT/prof5/kt_kernel_stats.csv | cut -c1-160 ;;
  profsimP)
    # per-rank kernel tables of the exchange mode at P in $SIMP (default 2 4 8), configs in
    # $SIMC (default c3 c5), simulated ranks one call at a time (MG_SIM_SERIAL)
    for C in ${SIMC:-c3 c5}; do
      for P in ${SIMP:-2 4 8}; do
        MG_SIM_SERIAL=1 timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profsim${P}_$C -o kt -- python3 bench.py --config $C --sim-world $P --multi exchange --steps 2 --no-cpu-baseline --no-ingest --opt layout_scratch=0 $SIMOPTS > $OUT/profsim${P}_${C}_bench.json 2> $OUT/profsim${P}_${C}_bench.err
        rc=$?; echo "profsim $P $C rc=$rc"; [ $rc -ne 0 ] && break 2
        python3 tools/rank_table.py $OUT/profsim${P}_$C/kt_kernel_stats.csv $P 4 "$C exchange-sim" > $OUT/profsim${P}_${C}_ranks.md
        tail -3 $OUT/profsim${P}_${C}_ranks.md
      done
    done ;;
  wattr)
    # C5 k_scan<INDEX> write attribution: WRITE_SIZE of the default build,
    # of the same build with no index inserts (option phase_limit=1), and of the 4-wave
    # spill-free variant (metagenomics_amd/lib/variants/scan_w4.so)
    for V in ${WATTR:-default noins w4}; do
      case $V in
        default) o=""; lib="" ;;
        noins) o="--opt phase_limit=1"; lib="" ;;
        w4) o=""; lib=$PWD/metagenomics_amd/lib/variants/scan_w4.so ;;
        *) o="--opt phase_limit=1"; lib=$PWD/metagenomics_amd/lib/variants/$V.so ;;  # diagnostics builds, inserts off
      esac
      MG_LIB=$lib timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $OUT/wattr_${WATTR_CONFIG:-c5}_$V -o p -- python3 bench.py --config ${WATTR_CONFIG:-c5} --steps 1 --warmup 0 --no-cpu-baseline --no-ingest --no-one-shot --no-d2h $o > $OUT/wattr_$V.log 2>&1
      rc=$?; echo "wattr $V rc=$rc"; [ $rc -ne 0 ] && break
      python3 tools/pmc_summary.py $OUT/wattr_${WATTR_CONFIG:-c5}_$V.json $OUT/wattr_${WATTR_CONFIG:-c5}_$V > /dev/null
      python3 -c "import json;d=json.load(open('$OUT/wattr_${WATTR_CONFIG:-c5}_$V.json'))['kernels'];[print('  ',k,round(v.get('WRITE_SIZE',0)/2**20,3),'GiB') for k,v in d.items() if k.startswith('k_scan') or k.startswith('k_probe')]"
    done ;;
  xhost)
    timeout -k 10 900 python -u -m pytest tests/test_xchg_host.py -x -v -m gpu --timeout 700 --timeout-method thread > $OUT/xhost_tests.log 2>&1
    rc=$?; echo "C++ exchange host tests rc=$rc"; grep -E "PASS|FAIL|Error" $OUT/xhost_tests.log | tail -30 ;;
  repro)
    make -s -C tools/micro over_heads_repro > $OUT/repro_build.log 2>&1 && timeout -k 10 120 tools/micro/over_heads_repro > $OUT/over_heads_repro.json 2>&1
    rc=$?; echo "over_heads repro rc=$rc"; cat $OUT/over_heads_repro.json ;;
  *) echo "unknown step $s"; rc=2 ;;
  esac
  if [ $rc -ne 0 ]; then tail -30 $OUT/*.err 2>/dev/null; exit $rc; fi
done
exit 0
