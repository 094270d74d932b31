# Round-4 GPU session: tests, bench in both arithmetics, a single-stream rocprofv3 trace of the
# bench's batch launch, and PMC of the launches bench.py's roofline blocks time (one counter group
# per run, never combined with tracing).  Every step has its own time limit; stops at the first failure.
#   TAG=name  SKIP_TESTS=1  SKIP_PMC=1  SKIP_BENCH=1  PMC_CONFIGS="dragon_1080 ..."  PMC_SPECS="fma:16 fma:1"
#   BENCH_ARGS="..."  SWEEP="bunny_640 ..." (bench.py --config for each, after the PMC)  REHEARSE="dragon_1080 ..."
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r04}; mkdir -p "$OUT"
step() { local t=$1; shift; local name=$1; shift; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-2} | cut -c1-400
         if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi; }
if [ -z "${SKIP_TESTS:-}" ]; then
  step 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
  step 900 pytest_gpu python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
fi
if [ -z "${SKIP_BENCH:-}" ]; then
step 300 bench_fma python bench.py ${BENCH_ARGS:-}
step 300 bench_exact python bench.py --arith exact --no-cpu-baseline ${BENCH_ARGS:-}
step 300 trace_batch rocprofv3 --kernel-trace --stats -d $OUT/trace_batch -o run -- python3 tools/batch_launch.py dragon_1080 fma 16 50
step 300 trace_step1 rocprofv3 --kernel-trace --stats -d $OUT/trace_step1 -o run -- python3 bench.py --streams 1 --steps 50 --warmup 5 --no-cpu-baseline --no-view0-only --no-roofline
fi
if [ -z "${SKIP_PMC:-}" ]; then
  P1="FETCH_SIZE TCC_REQ_sum GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
  P2="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR"
  P3="TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"
  for c in ${PMC_CONFIGS:-dragon_1080}; do
    for spec in ${PMC_SPECS:-fma:16 fma:1 exact:16 exact:1}; do
      set -- ${spec/:/ }; ar=$1; fr=$2
      suf=$([ "$fr" = 1 ] && echo "_solo_$ar" || echo "_batch${fr}_$ar")
      i=0
      for g in "$P1" "$P2" "$P3"; do
        i=$((i+1))
        step 240 pmc_${c}${suf}_p$i rocprofv3 --pmc $g --output-format csv -d $OUT/pmc/$c$suf/p$i -o run -- python3 tools/batch_launch.py $c $ar $fr 5
      done
      python3 tools/pmc_summary.py $c $OUT/pmc/$c$suf $OUT/pmc_summary.json $suf > /dev/null || exit 3
    done
  done
  # install the fresh counters in the tree's summary (on the box) so the sweep's roofline blocks read them
  python3 - "$OUT/pmc_summary.json" <<'PY' || exit 3
import json, sys
new = json.load(open(sys.argv[1]))
cur = json.load(open("profiles/pmc_summary.json"))
for cfg, kern in new.items():
    cur.setdefault(cfg, {}).update(kern)
json.dump(cur, open("profiles/pmc_summary.json", "w"), indent=1, sort_keys=True)
json.dump(cur, open(sys.argv[1].replace(".json", "_merged.json"), "w"), indent=1, sort_keys=True)
PY
fi
for c in ${SWEEP:-}; do
  steps=100; [ $c = proc_c5 ] && steps=20; [ $c = dragon_4096 ] && steps=50
  step 400 bench_$c python bench.py --config $c --steps $steps --warmup 5
done
for c in ${REHEARSE:-}; do
  step 400 rehearsal_$c python tools/scaling_rehearsal.py $c 20 16
done
exit 0
