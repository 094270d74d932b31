set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python tools/ab.py dragon_1080 30 ceres-raytracer_amd/libceres_hip.so ceres-raytracer_amd/variants/libceres_hip_sbvh2.so > gpurun_out/ab.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ab.log | tail -2
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/bench.log | tail -1
