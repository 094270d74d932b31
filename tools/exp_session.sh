set -u; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
make -C tools/probes 2>/dev/null >/dev/null || true
timeout -k 10 300 python tools/bvh_bench.py --config proc_c5 --reps 5 --host-reps 0 > gpurun_out/bvh.log 2>&1; echo bvh rc=$?; tail -1 gpurun_out/bvh.log | cut -c1-400
timeout -k 10 400 python tools/pipeline_bench.py proc_c5 > gpurun_out/pipe.log 2>&1; echo pipe rc=$?; tail -1 gpurun_out/pipe.log | cut -c1-600
