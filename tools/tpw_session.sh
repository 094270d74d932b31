# GPU session: tiles per wavefront in batches (CERES_TILES_PER_WAVE 2 / 4 / 8), in-process A/B,
# 16-frame batches over 8 streams, after the GPU parity tests of the default build.
set -u; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 3; }
tail -1 gpurun_out/pytest_gpu.log
BATCH=16 NFRAMES=128 ROUNDS=6 LIBS="ceres-raytracer_amd/libceres_hip.so ceres-raytracer_amd/variants/libceres_hip_tpw2.so ceres-raytracer_amd/variants/libceres_hip_tpw8.so" CONFIGS="${CONFIGS:-dragon_1080 bunny_1080 dragon_4096}" bash tools/ab_batch_session.sh || exit 3
