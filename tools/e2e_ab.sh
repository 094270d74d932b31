# Drop-in end-to-end per render<float>() call (tools/probes/dropin_bench, static.cpp-style caller of
# include/ceres/render.hpp), C3 and dragon 4096^2 (and C5 with C5=1), after the drop-in tests.
# ZC="1 0" A/Bs the zero-copy compacted readback (CERES_COMPACT_ZC).  Outputs under gpurun_out/$TAG.
set -u; cd "$GRAFT_REPO_ROOT"; OUT=gpurun_out/${TAG:-e2e_ab}; mkdir -p $OUT
A="data/dragon.obj --eye 0.0 -15.0 2.0 --dir 0.0 1.0 0.0 --up 0.0 0.0 1.0 --sun -50.0 -20.0 0.0 --rotate x 90.0"
if [ -n "${TESTS:-1}" ]; then
  timeout -k 10 600 python -u -m pytest ${TEST_FILES:-tests/test_gpu_readback.py tests/test_gpu_hardening.py} -m gpu -x -q --timeout 300 --timeout-method thread ${TEST_K:-} > $OUT/pytest.log 2>&1 || { tail -5 $OUT/pytest.log; exit 3; }
  tail -1 $OUT/pytest.log
fi
for r in ${ROUNDS:-1 2 3}; do for zc in ${ZC:-1}; do for sz in "1920 1080" "4096 4096"; do
  t=${sz/ /x}_zc${zc}_r$r
  CERES_COMPACT_ZC=$zc timeout -k 10 120 tools/probes/dropin_bench $A --size $sz --reps 50 --out $OUT/d.ppm > $OUT/dropin_$t.json 2>&1 || { cat $OUT/dropin_$t.json; exit 3; }
  echo "$t $(cat $OUT/dropin_$t.json) sha=$(sha256sum $OUT/d.ppm | cut -c1-16)"
done; done; done
if [ -n "${C5:-}" ]; then
  P="--proc 2237 --size 3840 2160 --eye 0.5 -0.4 0.6 --dir 0.0 0.9 -0.55 --up 0.0 0.0 1.0 --sun -50.0 -20.0 100.0"
  for b in dropin_bench dropin_bench_trust; do
    timeout -k 10 300 tools/probes/$b $P --reps 10 --out $OUT/c5.ppm > $OUT/${b}_c5.json 2>&1 || { cat $OUT/${b}_c5.json; exit 3; }
    echo "$b c5 $(cat $OUT/${b}_c5.json) sha=$(sha256sum $OUT/c5.ppm | cut -c1-16)"
  done
fi
rm -f $OUT/d.ppm $OUT/c5.ppm
