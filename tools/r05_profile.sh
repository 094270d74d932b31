# Round-5 profile session: for each launch bench.py's roofline blocks time (tools/batch_launch.py:
# config, arithmetic, frames per launch -- 16 = the bench step's batch of config-view copies, 1 =
# the solo frame), a single-stream rocprofv3 kernel trace (--kernel-trace --stats) and three PMC
# passes (one counter group per run, never combined with tracing; block limits per pass), then
# tools/pmc_summary.py into $OUT/pmc_summary.json and merged into profiles/pmc_summary.json on the
# box.  Every step has its own time limit; stops at the first failure.
#   TAG=name  SPECS="dragon_1080:fma:16 dragon_1080:fma:1 proc_c5:fma:1"  NO_PMC=1  NO_TRACE=1  BENCH_ARGS=".."
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05prof}; mkdir -p "$OUT"
step() { local t=$1; shift; local name=$1; shift; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-2} | cut -c1-400
         if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi; }
P1="FETCH_SIZE TCC_REQ_sum GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
P2="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR"
P3="TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"
for spec in ${SPECS:-dragon_1080:fma:16 dragon_1080:fma:1 proc_c5:fma:1}; do
  IFS=: read -r c ar fr <<< "$spec"
  suf=$([ "$fr" = 1 ] && echo "_solo_$ar" || echo "_batch${fr}_$ar")
  n=50; [ $c = proc_c5 ] && n=10
  if [ -z "${NO_TRACE:-}" ]; then
    step 300 trace_$c$suf rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$c$suf -o run -- python3 tools/batch_launch.py $c $ar $fr $n
  fi
  if [ -z "${NO_PMC:-}" ]; then
    i=0
    for g in "$P1" "$P2" "$P3"; do
      i=$((i+1))
      step 240 pmc_$c${suf}_p$i rocprofv3 --pmc $g --output-format csv -d $OUT/pmc/$c$suf/p$i -o run -- python3 tools/batch_launch.py $c $ar $fr 5
    done
    python3 tools/pmc_summary.py $c $OUT/pmc/$c$suf $OUT/pmc_summary.json $suf > /dev/null || exit 3
  fi
done
if [ -z "${NO_PMC:-}" ]; then
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
if [ -z "${NO_BENCH:-}" ]; then step 300 bench python bench.py ${BENCH_ARGS:-}; fi
exit 0
