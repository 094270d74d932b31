set -u; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for p in "--double" ""; do
  timeout -k 10 120 ceres-raytracer_amd/render data/dragon.obj --rotate x 90 $p --bench 50 --json -o /tmp/d.ppm > gpurun_out/cli$p.log 2>&1 || exit 1
  tail -1 gpurun_out/cli$p.log
done
AB_STREAMS=8 AB_BATCH=4 AB_FRAMES=32 SKIP_TESTS=1 CONFIGS="dragon_1080 bunny_1080" ROUNDS=12 bash tools/session_ab.sh
