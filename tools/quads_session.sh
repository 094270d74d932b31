# GPU session: lane -> pixel mapping of the fused kernel's 8x8 tile (row-major vs Morton /
# 2x2 quads, CERES_LANE_QUADS), in-process A/B: solo frames and 16-frame batches x 8 streams.
set -u; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
SOLO=1 BATCH=16 NFRAMES=128 ROUNDS=6 LIBS="ceres-raytracer_amd/libceres_hip.so ceres-raytracer_amd/variants/libceres_hip_quads.so" CONFIGS="${CONFIGS:-dragon_1080 bunny_1080 dragon_4096 proc_c5}" bash tools/ab_batch_session.sh || exit 3
