# GPU session: refresh the rocprofv3 --pmc summary of every config bench reports (C1 included), install
# it as profiles/pmc_summary.json on the box (a copy comes back as gpurun_out/pmccfg/pmc_summary_new.json,
# to be committed), then the per-config bench sweep, whose roofline blocks read that summary, then a
# rocprofv3 kernel trace + stats of the default bench command.  Every GPU step has its own time limit.
set -u; cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
CONFIGS="bunny_640 bunny_1080_primary bunny_1080 dragon_1080 dragon_4096 proc_c5" bash tools/pmc_configs_session.sh || exit 3
cp gpurun_out/pmccfg/pmc_summary_new.json profiles/pmc_summary.json || exit 3
REHEARSE=" " bash tools/sweep_session.sh || exit 3
mkdir -p gpurun_out/final
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/trace -o run -- python3 bench.py > gpurun_out/final/bench_under_rocprof.log 2>&1 || { tail -5 gpurun_out/final/bench_under_rocprof.log; exit 3; }
grep -v amdgpu.ids gpurun_out/final/bench_under_rocprof.log | tail -1 | cut -c1-200
