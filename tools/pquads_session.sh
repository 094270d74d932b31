# GPU session: Morton lane order in the primary-only kernel (CERES_PRIMARY_LANE_QUADS), GPU parity
# tests, then in-process A/B on C2 (bunny 1080p primary only): solo frames and 16-frame batches.
set -u; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 3; }
tail -1 gpurun_out/pytest_gpu.log
SOLO=1 BATCH=16 NFRAMES=128 ROUNDS=8 LIBS="ceres-raytracer_amd/libceres_hip.so ceres-raytracer_amd/variants/libceres_hip_prow.so" CONFIGS="bunny_1080_primary" bash tools/ab_batch_session.sh || exit 3
SOLO=1 BATCH=16 NFRAMES=128 ROUNDS=8 LIBS="ceres-raytracer_amd/variants/libceres_hip_prow.so ceres-raytracer_amd/libceres_hip.so" CONFIGS="bunny_1080_primary" bash tools/ab_batch_session.sh || exit 3
