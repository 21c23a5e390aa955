#!/bin/bash
# Round-6 final captures on the final build, in three GPU calls (each step timed
# and chained: the first failure ends the call).
#   A: full -m gpu suite, smoke, C3 PMC passes, C3 bench (with that PMC), C3 kernel trace, one RCCL rank
#   B: C5 PMC passes, C5 bench (with that PMC), C5 simulated P = 8 exchange table
#   C: C3 simulated per-rank tables: exchange P = 2/4/8, bucket and replicated P = 2/4/8
set -o pipefail
T=${TAG:-r06f}
OUT=gpurun_out/$T
mkdir -p $OUT
# run MODE: the gpu_run.sh step, its output kept and shown; fails unless it printed an
# " rc=0" and no nonzero rc
run() {
  bash tools/gpu_run.sh $T "$1" > $OUT/step_$1.log 2>&1
  cat $OUT/step_$1.log
  grep -E " rc=0" $OUT/step_$1.log > /dev/null && ! grep -E " rc=[1-9]" $OUT/step_$1.log > /dev/null
}
case "$1" in
  A)
    run tests && ! grep -qE "[0-9]+ (failed|error)" $OUT/gpu_tests.log &&
    run smoke &&
    run pmc && test -f $OUT/pmc_summary.json &&
    timeout -k 10 600 python -u bench.py --pmc $OUT/pmc_summary.json > $OUT/bench.json 2> $OUT/bench.err &&
    echo "bench ok" && head -c 600 $OUT/bench.json && echo &&
    run prof &&
    run xchg1 ;;
  B)
    run pmc5 && test -f $OUT/pmc5_summary.json &&
    timeout -k 10 600 python -u bench.py --config c5 --no-ingest --pmc $OUT/pmc5_summary.json > $OUT/bench_c5.json 2> $OUT/bench_c5.err &&
    echo "bench c5 ok" && head -c 600 $OUT/bench_c5.json && echo &&
    SIMC=c5 SIMP=8 run profsimP ;;
  C)
    SIMC=c3 SIMP="2 4 8" run profsimP &&
    SIMP="2 4 8" run simbkt &&
    run simrep ;;
  *) echo "usage: r06_final.sh A|B|C"; exit 2 ;;
esac
