# A/B of library builds (LIBS = space-separated .so paths) on CONFIGS; optional rocprof pass (PROF=1).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
LIBS=${LIBS:-ceres-raytracer_amd/libceres_hip.so}
for cfg in ${CONFIGS:-dragon_1080}; do
  timeout -k 10 300 python tools/ab.py $cfg ${ROUNDS:-20} $LIBS > gpurun_out/ab_$cfg.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/ab_$cfg.log | tail -3
  if [ $rc -ne 0 ]; then exit $rc; fi
done
if [ -n "${PROF:-}" ]; then
  for l in $LIBS; do
    tag=$(basename $l .so)
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ab/$tag -o run -- python3 tools/ab.py dragon_1080 10 $l > gpurun_out/prof_ab_$tag.log 2>&1 || exit 1
    cut -d, -f1-4 gpurun_out/prof_ab/$tag/run_kernel_stats.csv | head -5
  done
fi
