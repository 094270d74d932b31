set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in ${CONFIGS:-dragon_1080}; do
  timeout -k 10 300 python tools/ab.py $cfg ${ROUNDS:-20} ${VARIANTS:-wave twopass frame} > gpurun_out/ab_$cfg.log 2>&1; rc=$?
  grep -v amdgpu.ids gpurun_out/ab_$cfg.log | tail -3
  if [ $rc -ne 0 ]; then exit $rc; fi
done
if [ -n "${PROF:-}" ]; then
  for v in ${VARIANTS:-wave}; do
    kern=${v%%:*}; tpw=${v#*:}; [ "$tpw" = "$v" ] && tpw=1
    CERES_KERNEL=$kern CERES_TPW=$tpw timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ab/$kern$tpw -o run -- python3 tools/ab.py dragon_1080 10 $v > gpurun_out/prof_ab_$kern$tpw.log 2>&1 || exit 1
    cut -d, -f1-4 gpurun_out/prof_ab/$kern$tpw/run_kernel_stats.csv | head -4
  done
fi
