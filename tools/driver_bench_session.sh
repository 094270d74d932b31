# GPU session: the GPU parity suite, then bench.py exactly as the driver runs it (--steps 20
# --warmup 5) three times plus the default (200-step) run; each step under its own time limit.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-3} "gpurun_out/$name.log"; if [ $rc -gt 1 ]; then echo "STOP after $name"; exit $rc; fi; return 0; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  step 900 pytest_gpu python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
fi
for i in 1 2 3; do
  step 300 drv$i python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_EXTRA:-}
done
step 400 bench python bench.py ${BENCH_EXTRA:-}
