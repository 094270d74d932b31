# rocprofv3 session: kernel trace + stats of bench.py, then separate PMC passes (one counter
# group per run, never combined with -s/-r/tracing domains).  Outputs under gpurun_out/prof/.
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof_${CFG:-dragon_1080}
mkdir -p $OUT
# --streams 1 --frames 1: every launch one serialised frame, so the trace mean per kernel is the solo
# one-frame duration bench.py prices
CFG=${CFG:-dragon_1080}
BENCH="bench.py --config $CFG --steps ${STEPS:-50} --warmup 5 --no-cpu-baseline --streams 1 --frames 1"
step() { local t=$1; shift; local name=$1; shift; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 "$OUT/$name.log"; if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi; }
step 120 list rocprofv3 -L
step 400 trace rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $BENCH
step 400 pmc_fetch rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-roofline --streams 1 --frames 1
step 400 pmc_write rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-roofline --streams 1 --frames 1
step 400 pmc_sq rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU --output-format csv -d $OUT/pmc_sq -o run -- python3 bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-roofline --streams 1 --frames 1
step 400 pmc_sq2 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR --output-format csv -d $OUT/pmc_sq2 -o run -- python3 bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-roofline --streams 1 --frames 1
step 400 pmc_l2 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_l2 -o run -- python3 bench.py --config $CFG --steps 10 --warmup 2 --no-cpu-baseline --no-roofline --streams 1 --frames 1
python3 tools/pmc_summary.py $CFG $OUT $OUT/pmc_summary.json > /dev/null && echo summary ok
