# bench.py itself, alternating library builds (CERES_LIB), ROUNDS rounds: the driver's command
# (--steps 20 --warmup 5) and the default 200-step run.  LIBS = space-separated .so paths.
set -u; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in $(seq ${ROUNDS:-2}); do
  for l in $LIBS; do
    for a in "--steps 20 --warmup 5" ""; do
      CERES_LIB=$PWD/$l timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline $a ${BENCH_EXTRA:-} > gpurun_out/bab.log 2>&1 || { tail -3 gpurun_out/bab.log; exit 3; }
      python -c "import json,sys; d=json.loads(open('gpurun_out/bab.log').read().strip().splitlines()[-1]); print(sys.argv[1], sys.argv[2], d['value'], d['parity'])" "$(basename $l)" "[$a]"
    done
  done
done
