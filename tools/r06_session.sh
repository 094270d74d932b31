# Round-6 GPU session: every step under its own time limit, chained so the first failure stops
# the run (no GPU step after a fault or a timeout).  Steps (STEPS="..." picks a subset):
#   tests   pytest -m gpu (thread timeouts, one process)
#   bench   bench.py default line (C3) -> $OUT/bench_dragon_1080.log
#   trace   rocprofv3 --kernel-trace of bench.py's own timed loop (tools/step_trace.py summary)
#   l1      the vector-L1 calibration probe under rocprofv3 --pmc (three load shapes)
#   ab      tools/ab.py A/B of $AB_LIBS in the throughput regime (16-frame batches x 8 streams)
#   abs     tools/ab.py A/B of $AB_LIBS, single frames
#   sweep   bench.py on every BASELINE config ($SWEEP)
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06}; mkdir -p "$OUT"
step() { local t=$1; shift; local name=$1; shift; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-3} | cut -c1-600
         if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi; }
has() { case " ${STEPS:-tests bench} " in *" $1 "*) return 0;; esac; return 1; }
if has tests; then
  step 900 pytest_gpu python -u -m pytest ${PYTEST_FILES:-tests} -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_K:-}
fi
if has bench; then
  step 400 bench_dragon_1080 python bench.py ${BENCH_ARGS:-}
fi
if has trace; then
  step 400 steptrace_bench rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/steptrace -o run -- \
      python3 bench.py --steps ${TRACE_STEPS:-20} --warmup 5 --no-orbit --no-roofline --no-cpu-baseline ${TRACE_ARGS:-}
  python3 tools/step_trace.py $OUT/steptrace $OUT/steptrace_bench.log $OUT/step_trace_dragon_1080_fma.json || exit 3
fi
if has l1; then
  for m in 0 1 2; do
    step 120 l1_time_$m tools/probes/l1_peak $m 4096
    step 120 l1_pmc_$m rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE --output-format csv \
        -d $OUT/l1/m$m -o run -- tools/probes/l1_peak $m 4096
  done
fi
if has ab; then
  for c in ${AB_CFGS:-dragon_1080 proc_c5}; do
    v=""; [ $c = proc_c5 ] && v=1
    AB_STREAMS=8 AB_BATCH=16 AB_FRAMES=${AB_FRAMES:-16} AB_VIEW0=$v step 600 ab_batch_$c python tools/ab.py $c ${AB_ROUNDS:-7} $AB_LIBS
  done
fi
if has abs; then
  for c in ${ABS_CFGS:-dragon_1080 proc_c5}; do
    step 600 ab_solo_$c python tools/ab.py $c ${ABS_ROUNDS:-15} $AB_LIBS
  done
fi
if has wr; then
  # DRAM write bytes of one 16-frame batch launch per library ($WR_LIBS), rocprofv3 --pmc WRITE_SIZE
  for lib in ${WR_LIBS:-ceres-raytracer_amd/libceres_hip.so}; do
    t=$(basename $lib .so)
    for c in ${WR_CFGS:-dragon_1080}; do
      CERES_LIB=$lib step 240 wr_${c}_$t rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv \
          -d $OUT/wr/${c}_$t -o run -- python3 tools/batch_launch.py $c fma 16 5
    done
  done
fi
if has sweep; then
  for c in ${SWEEP:-bunny_640 bunny_1080_primary bunny_1080 dragon_4096 proc_c5}; do
    step 600 bench_$c python bench.py --config $c ${SWEEP_ARGS:-}
  done
fi
exit 0
