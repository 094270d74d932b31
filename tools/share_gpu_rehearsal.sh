# Multi-rank bench rehearsal on a one-GPU box: N ranks share device 0 (CERES_BENCH_SHARE_GPU=1)
# (RCCL refuses two ranks on one device: the collectives run over gloo here).  Exercises the N > 1 code path of bench.py (all-to-all frame exchange, step
# streams, assembly, barrier/max timing); the numbers are NOT scaling numbers (one GPU).
set -u; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/share; export TMPDIR=/tmp
for N in ${NLIST:-2}; do
  for C in ${COLLECT:-exchange}; do
    CERES_BENCH_SHARE_GPU=1 CERES_BENCH_BACKEND=${BACKEND:-gloo} timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
      --master-addr 127.0.0.1 --master-port $((29500 + N)) bench.py --gpus $N --steps 40 --warmup 5 --collect $C \
      > gpurun_out/share/n${N}_$C.log 2>&1
    rc=$?; echo "N=$N $C rc=$rc"; grep -v amdgpu gpurun_out/share/n${N}_$C.log | tail -3 | cut -c1-400
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
