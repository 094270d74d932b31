# rocprofv3 --pmc passes over solo frames (tools/ab.py <cfg> 5: the launch bench.py's roofline
# times) for every config bench reports, one counter group per run (never combined with tracing),
# summarised per config into profiles/pmc_summary.json by tools/pmc_summary.py.
#   CONFIGS="..." (default: C2, bunny full, C3, C4 one GPU, C5 one GPU)   outputs: gpurun_out/pmccfg$SUFFIX/
#   LIB=path/to/libceres_hip_x.so: profile that build instead of the in-tree one (SUFFIX names the run)
set -u; cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/pmccfg${SUFFIX:-}; mkdir -p $OUT
P1="FETCH_SIZE TCC_REQ_sum GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES"
P2="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_WR"
P3="TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"
for c in ${CONFIGS:-bunny_1080_primary bunny_1080 dragon_1080 dragon_4096 proc_c5}; do
  i=0
  for g in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $g --output-format csv -d $OUT/$c/p$i -o run -- python3 tools/ab.py $c 5 ${LIB:-} > $OUT/$c.p$i.log 2>&1; rc=$?
    echo "$c pass $i rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $OUT/$c.p$i.log; exit $rc; fi
  done
  python3 tools/pmc_summary.py $c $OUT/$c $OUT/pmc_summary.json > /dev/null || exit 3
done
cp $OUT/pmc_summary.json $OUT/pmc_summary_new.json
