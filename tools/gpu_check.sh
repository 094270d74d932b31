# GPU check session: smoke(), the -m gpu parity suite, then optional A/B rounds against a
# variant build and a default bench.py run.  Every GPU step has its own time limit and the
# session stops at the first failure.  Outputs under gpurun_out/$TAG/.
#   TAG=name  AB="cfg ..." (configs for tools/ab.py, solo and 16-frame batches x 8 streams)
#   AB_LIBS="ceres-raytracer_amd/libceres_hip.so ceres-raytracer_amd/variants/libceres_hip_x.so"
#   AB_MODES="solo batch" (default both)  SKIP_TESTS=1  BENCH_ARGS="--steps 20 --warmup 5"  EXTRA="cmd" (one more command, 300 s)
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-check}; mkdir -p "$OUT"
step() { local t=$1; shift; local name=$1; shift; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?
         echo "$name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -${TAILN:-2} | cut -c1-600
         if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi; }
if [ -z "${SKIP_TESTS:-}" ]; then
  step 300 smoke python -c "import __graft_entry__ as g; g.smoke()"
  step 600 pytest_gpu python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
fi
M="${AB_MODES:-solo batch}"
for c in ${AB:-}; do
  [ "$M" != "${M/solo/}" ] && step 300 ab_solo_$c python tools/ab.py $c ${AB_ROUNDS:-20} ${AB_LIBS:-}
  [ "$M" != "${M/batch/}" ] && AB_STREAMS=8 AB_FRAMES=16 AB_BATCH=16 step 300 ab_batch_$c python tools/ab.py $c ${AB_ROUNDS:-8} ${AB_LIBS:-}
done
if [ -n "${EXTRA:-}" ]; then step 300 extra bash -c "$EXTRA"; fi
if [ -z "${NO_BENCH:-}" ]; then step 300 bench python bench.py ${BENCH_ARGS:-}; fi
exit 0
