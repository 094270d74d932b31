set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python tools/wave_diag.py dragon_1080 5 > gpurun_out/diag.log 2>&1; rc=$?; cat gpurun_out/diag.log | grep -v amdgpu.ids; exit $rc
