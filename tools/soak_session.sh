# Stability: GPU tests once, then the default bench three times (variance across runs).
set -u; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/soak; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/soak/pytest.log 2>&1 || { tail -20 gpurun_out/soak/pytest.log; exit 1; }
tail -1 gpurun_out/soak/pytest.log
for i in 1 2 3; do
  timeout -k 10 300 python bench.py > gpurun_out/soak/bench_$i.log 2>&1 || exit 1
  grep '^{' gpurun_out/soak/bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($i, d['value'], d['ms_per_step'], d['roofline']['mean_launch_ms'], d['roofline']['frac'], d['cpu_baseline']['value'], all(d['parity'].values()))"
done
