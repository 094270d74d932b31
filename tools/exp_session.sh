set -u; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
run() { timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline "$@" > gpurun_out/e.log 2>&1 || { tail -3 gpurun_out/e.log; exit 3; }; python -c "import json,sys; d=json.loads(open('gpurun_out/e.log').read().strip().splitlines()[-1]); print(sys.argv[1:], d['value'], d['ms_per_step'])" "$@"; }
for r in 1 2; do
run --steps 20 --warmup 5
run --steps 20 --warmup 5 --frames-per-gpu 16
run --steps 20 --warmup 5 --streams 4
run --steps 20 --warmup 5 --streams 16
run --steps 20 --warmup 5 --frames-per-gpu 4 --streams 16
done
