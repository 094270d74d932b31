set -u; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
CERES_LIB=$PWD/ceres-raytracer_amd/variants/libceres_hip_pk1.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scene.py -q -x -k "not dropin" --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -2 gpurun_out/t.log; [ $rc -ne 0 ] && exit $rc
SOLO=1 LIBS="ceres-raytracer_amd/libceres_hip.so ceres-raytracer_amd/variants/libceres_hip_pk1.so" CONFIGS="dragon_1080 bunny_1080 dragon_4096 proc_c5" bash tools/ab_batch_session.sh
