# PMC passes for the 4-frame batch launch (bench.py --frames 4 --streams 1; rocprofv3 --pmc
# serialises dispatches anyway).  Outputs under gpurun_out/pmcb/.
set -u; cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/pmcb; mkdir -p $OUT
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-roofline --streams 1 --frames 4 --config ${CFG:-dragon_1080}"
step() { local name=$1; shift; timeout -k 10 300 "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && { tail -3 $OUT/$name.log; exit $rc; }; return 0; }
step sq rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU --output-format csv -d $OUT/pmc_sq -o run -- python3 $B
step sq2 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR --output-format csv -d $OUT/pmc_sq2 -o run -- python3 $B
step l2 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_l2 -o run -- python3 $B
step trace rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $B
python3 tools/pmc_summary.py ${CFG:-dragon_1080} $OUT $OUT/pmc_summary.json > /dev/null && echo summary ok
