# GPU parity tests on the in-tree build, then an in-process A/B of LIBS (default: every variant).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
fi
LIBS=${LIBS:-"ceres-raytracer_amd/libceres_hip.so $(ls ceres-raytracer_amd/variants/*.so)"}
for cfg in ${CONFIGS:-dragon_1080}; do
  timeout -k 10 400 python tools/ab.py $cfg ${ROUNDS:-30} $LIBS > gpurun_out/ab_$cfg.log 2>&1 || { tail -5 gpurun_out/ab_$cfg.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/ab_$cfg.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); [print(d['config'], k, v) for k,v in d['results'].items()]"
done
