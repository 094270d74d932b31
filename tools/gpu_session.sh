# GPU session: smoke, GPU parity tests (both kernel variants), bench (both variants).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log"; if [ $rc -gt 1 ]; then echo "STOP after $name"; exit $rc; fi; return 0; }
step 400 smoke python -c "import __graft_entry__ as g; g.smoke()"
step 900 pytest_gpu python -m pytest tests -m gpu -q -x
CERES_KERNEL=twopass step 900 pytest_gpu_twopass python -m pytest tests -m gpu -q -x
step 400 bench python bench.py --steps 100 --warmup 10 --no-cpu-baseline
CERES_KERNEL=twopass step 400 bench_twopass python bench.py --steps 100 --warmup 10 --no-cpu-baseline
