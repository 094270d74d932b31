# GPU session for a tile-order change: GPU parity tests, in-process A/B against the
# interleaved order (16-frame batches), then bench.py on the configs it affects.
set -u; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 3; }
tail -1 gpurun_out/pytest_gpu.log
BATCH=16 NFRAMES=128 ROUNDS=5 LIBS="ceres-raytracer_amd/libceres_hip.so ceres-raytracer_amd/variants/libceres_hip_inter.so" CONFIGS="dragon_1080 dragon_4096 proc_c5" bash tools/ab_batch_session.sh || exit 3
CONFIGS="dragon_4096 proc_c5 dragon_1080" REHEARSE=" " bash tools/sweep_session.sh
