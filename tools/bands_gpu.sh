set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/r06ab; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
CERES_BENCH_SHARE_GPU=1 CERES_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --collect bands --steps 5 --warmup 2 --no-orbit --no-roofline --no-cpu-baseline > $OUT/bench_n2_bands.log 2>&1; rc=$?
grep '^{"metric"' $OUT/bench_n2_bands.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['config']['collect'], d['parity'], d.get('partition_alt',{}).get('collect'), d.get('partition_alt',{}).get('value'))" || tail -20 $OUT/bench_n2_bands.log
exit $rc
