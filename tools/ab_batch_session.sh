# A/B of library builds (LIBS) in one process per config (tools/ab.py): solo frames (SOLO=1) and
# the throughput regime (8-frame batches round-robin over 8 streams).  Prints median ms per frame.
set -u; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
L=${LIBS:-ceres-raytracer_amd/libceres_hip.so}
summ() { grep -v amdgpu.ids $1 | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config'], '$2', {k[12:-3]: v['median_ms'] for k, v in d['results'].items()}, all(v['parity'] for v in d['results'].values()))"; }
for c in ${CONFIGS:-dragon_1080 bunny_1080}; do
  if [ "${SOLO:-0}" = 1 ]; then
  timeout -k 10 300 python tools/ab.py $c ${ROUNDS:-20} $L > gpurun_out/abs_$c.log 2>&1 || { tail -5 gpurun_out/abs_$c.log; exit 3; }
  summ gpurun_out/abs_$c.log solo
  fi
  AB_STREAMS=8 AB_BATCH=${BATCH:-8} AB_FRAMES=${NFRAMES:-64} timeout -k 10 300 python tools/ab.py $c ${ROUNDS:-8} $L > gpurun_out/ab_$c.log 2>&1 || { tail -5 gpurun_out/ab_$c.log; exit 3; }
  summ gpurun_out/ab_$c.log batch${BATCH:-8}x8
done
