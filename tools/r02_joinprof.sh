# join path diagnostics: phase split, variant A/B, SQ counters of the scan and the join
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r02f}
mkdir -p $O
timeout -k 10 300 python -u tools/phase_sweep.py > $O/phases_join.log 2>&1 || exit 1
MG_VARIANTS='[{}, {"join":0}, {}, {"join":0}]' timeout -k 10 300 python -u tools/variant_sweep.py > $O/sweep.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --kernel-trace --output-format csv -d $O/pmc1 -o p -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ingest > $O/pmc1.log 2>&1 || exit 1
grep phase $O/phases_join.log; grep opts $O/sweep.log
python3 tools/pmc_summary.py $O/pmc_summary.json $O/pmc1 > /dev/null; python3 - <<'PY' $O
import json,sys
d=json.load(open(sys.argv[1]+"/pmc_summary.json"))
for k,v in d.get("kernels",{}).items():
    if any(x in k for x in ("k_join","k_scan","onesweep","histogram")):
        c=v; wc=c.get("SQ_WAVE_CYCLES",1) or 1
        print(k[-60:], "waves", c.get("SQ_WAVES"), "busy", c.get("SQ_BUSY_CYCLES"), "wait%", round(100*c.get("SQ_WAIT_ANY",0)/wc,1),
              "active%", round(100*c.get("SQ_ACTIVE_INST_ANY",0)/wc,1), "waitinst%", round(100*c.get("SQ_WAIT_INST_ANY",0)/wc,1),
              "valu", c.get("SQ_INSTS_VALU"), "lds", c.get("SQ_INSTS_LDS"))
PY
