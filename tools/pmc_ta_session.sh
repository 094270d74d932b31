# PMC passes for the texture-address / L1 path (TA, TD, TCP blocks) on the 8-frame batch launch
# (bench.py --frames 8 --streams 1); counter availability listed first.  Outputs under gpurun_out/pmcta/.
set -u; cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/pmcta; mkdir -p $OUT
B="bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-roofline --streams 1 --frames 8 --config ${CFG:-dragon_1080}"
timeout -k 10 120 rocprofv3 --list-avail > $OUT/avail.txt 2>&1; echo "list rc=$?"
grep -oE '\b(TA|TD|TCP)_[A-Za-z0-9_]+' $OUT/avail.txt | sort -u > $OUT/avail_ta.txt || true
wc -l $OUT/avail_ta.txt
pass() { local name=$1; shift; timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 $B > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && { tail -3 $OUT/$name.log; exit $rc; }; return 0; }
pass ta TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum GRBM_GUI_ACTIVE
pass td TD_TD_BUSY_sum TD_TC_STALL_sum
pass tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD
