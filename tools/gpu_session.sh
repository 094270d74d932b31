# GPU session: smoke, GPU parity tests, bench (N=1), each step under its own time limit.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1; shift; local name=$1; shift; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-4} "gpurun_out/$name.log"; if [ $rc -gt 1 ]; then echo "STOP after $name"; exit $rc; fi; return 0; }
step 400 smoke python -c "import __graft_entry__ as g; g.smoke()"
step 900 pytest_gpu python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
step 400 bench python bench.py
step 400 bench_f1 python bench.py --steps 200 --warmup 10 --frames 1 --no-cpu-baseline --no-roofline
