# GPU session after making the Morton lane mapping the default: GPU parity tests, the A/B reversed
# (default vs the row-major variant), then the default bench command.
set -u; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 3; }
tail -1 gpurun_out/pytest_gpu.log
SOLO=1 BATCH=16 NFRAMES=128 ROUNDS=6 LIBS="ceres-raytracer_amd/libceres_hip.so ceres-raytracer_amd/variants/libceres_hip_rowmajor.so" CONFIGS="${CONFIGS:-dragon_1080 bunny_1080 dragon_4096 proc_c5}" bash tools/ab_batch_session.sh || exit 3
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || { tail -5 gpurun_out/bench.log; exit 3; }
grep -v amdgpu.ids gpurun_out/bench.log | tail -1 | cut -c1-200
