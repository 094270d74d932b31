# Round-5 GPU session: smoke, the -m gpu suite on the default build and (optionally) on a variant
# build, then A/B of variant builds (tools/ab.py, solo and 16-frame batches x 8 streams).
# Every GPU step has its own time limit; the session stops at a fault, abort or time limit.
#   TAG=name  SKIP_TESTS=1  VARIANT_TEST=lib.so (suite again with CERES_LIB=lib.so; failures are
#   recorded, not fatal)  AB="cfg ..."  AB_LIBS="a.so b.so ..."  AB_MODES="solo batch"
#   AB_ROUNDS_SOLO=30 AB_ROUNDS_BATCH=12  EXTRA="cmd"  BENCH_ARGS="..."  NO_BENCH=1
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r05}; mkdir -p "$OUT"
step() { local fatal=$1; shift; local t=$1; shift; local name=$1; shift
         timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-2} | cut -c1-600
         case $rc in 0) ;; 1) [ "$fatal" = soft ] || { echo "STOP after $name"; exit 1; } ;;
                     *) echo "STOP after $name (rc $rc)"; exit $rc ;; esac; }
if [ -z "${SKIP_TESTS:-}" ]; then
  step hard 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
  step hard 600 pytest_gpu python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
fi
if [ -n "${VARIANT_TEST:-}" ]; then
  CERES_LIB=$VARIANT_TEST step soft 600 pytest_gpu_variant python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread
fi
M="${AB_MODES:-solo batch}"
for c in ${AB:-}; do
  [ "$M" != "${M/solo/}" ] && step hard 400 ab_solo_$c python tools/ab.py $c ${AB_ROUNDS_SOLO:-30} ${AB_LIBS:-}
  [ "$M" != "${M/batch/}" ] && AB_STREAMS=8 AB_FRAMES=16 AB_BATCH=16 AB_VIEW0=${AB_VIEW0:-0} \
      step hard 400 ab_batch_$c python tools/ab.py $c ${AB_ROUNDS_BATCH:-12} ${AB_LIBS:-}
done
if [ -n "${EXTRA:-}" ]; then step hard 400 extra bash -c "$EXTRA"; fi
if [ -z "${NO_BENCH:-}" ]; then step hard 300 bench python bench.py ${BENCH_ARGS:-}; fi
exit 0
