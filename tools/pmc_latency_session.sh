# PMC passes on the 8-frame batch launch (bench.py --frames 8 --streams 1): outstanding-instruction
# levels (Little's law: mean latency = level / instructions), TA FIFO back-pressure, issue-stall
# split, LDS conflicts, TA/TD/TCP busy.  Outputs under gpurun_out/pmclat/.
set -u; cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/pmclat; mkdir -p $OUT
B="bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-roofline --streams 1 --frames 8 --config ${CFG:-dragon_1080}"
pass() { local name=$1; shift; timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 $B > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; [ $rc -ne 0 ] && { tail -3 $OUT/$name.log; exit $rc; }; return 0; }
pass lvl SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAVES
pass act SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS
pass misc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_IFETCH SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
pass ta TA_TA_BUSY_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum
pass l2 TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum SQ_INSTS_VMEM_RD SQ_INSTS_SMEM_NORM SQ_INST_CYCLES_VMEM_RD
