# End-of-round GPU session: smoke, GPU parity tests, the per-config bench sweep (REHEARSE=" " skips
# the scaling rehearsal), then rocprofv3 kernel trace + stats of the default bench command.
set -u; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/final; export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1 || { tail -5 gpurun_out/final/smoke.log; exit 3; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/final/pytest_gpu.log; exit 3; }
tail -1 gpurun_out/final/pytest_gpu.log
REHEARSE=" " bash tools/sweep_session.sh || exit 3
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/trace -o run -- python3 bench.py > gpurun_out/final/bench_under_rocprof.log 2>&1 || { tail -5 gpurun_out/final/bench_under_rocprof.log; exit 3; }
grep -v amdgpu.ids gpurun_out/final/bench_under_rocprof.log | tail -1 | cut -c1-200
