# Round-6 final profile of the current build, in two calls (each under gpurun's 20-minute limit):
#   PART=prof : single-stream kernel traces + three PMC passes of every config's 16-frame batch launch
#               and solo frame (tools/r05_profile.sh), merged into profiles/pmc_summary.json on the box
#               (gpurun_out/$TAG/prof/pmc_summary_merged.json comes back)
#   PART=bench: smoke, the step trace of bench.py's timed loop (copied to profiles/r06/ on the box so the
#               sweep's C3 line carries it), then bench.py on every BASELINE config
# Every step has its own time limit; stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=${TAG:-r06final}
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
if [ "${PART:-prof}" = prof ]; then
  TAG=$TAG/prof NO_BENCH=1 SPECS="${SPECS:-dragon_1080:fma:16 dragon_1080:fma:1 bunny_1080:fma:16 bunny_1080:fma:1 bunny_1080_primary:fma:16 bunny_1080_primary:fma:1 bunny_640:fma:16 bunny_640:fma:1 dragon_4096:fma:16 dragon_4096:fma:1 proc_c5:fma:16 proc_c5:fma:1}" \
    bash tools/r05_profile.sh || exit $?
  exit 0
fi
if [ -n "${PMC_JSON:-}" ]; then cp "$PMC_JSON" profiles/pmc_summary.json; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 3; }
tail -1 $OUT/smoke.log
TAG=$TAG STEPS=trace bash tools/r06_session.sh || exit $?
cp $OUT/step_trace_dragon_1080_fma.json profiles/r06/step_trace_dragon_1080_fma.json
for c in ${SWEEP:-dragon_1080 bunny_640 bunny_1080_primary bunny_1080 dragon_4096 proc_c5}; do
  timeout -k 10 600 python bench.py --config $c > $OUT/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -5 $OUT/bench_$c.log; exit 3; }
  grep '^{"metric"' $OUT/bench_$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['ms_per_step'], d['roofline']['bound'], d['roofline']['frac'], d['roofline_step']['bound'], d['roofline_step']['frac'], d['parity'].get('all_frames_match_reference'))"
done
# the N > 1 path with the band partition: 2 ranks sharing the GPU over gloo (not a scaling number)
CERES_BENCH_SHARE_GPU=1 CERES_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --collect bands --steps 5 --warmup 2 --no-orbit \
    --no-roofline --no-cpu-baseline > $OUT/bench_n2_bands.log 2>&1 || { tail -20 $OUT/bench_n2_bands.log; exit 3; }
grep '^{"metric"' $OUT/bench_n2_bands.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('n2 bands', d['value'], d['config']['collect'], d['parity']['all_frames_match_reference'], d.get('partition_alt',{}).get('collect'))"
exit 0
