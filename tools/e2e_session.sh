# Drop-in boundary cost per call (render.hpp:86-89 as static.cpp / anim.cpp call it): the
# static.cpp-style tools/probes/dropin_bench through include/ceres/render.hpp (host float
# framebuffer) and ./render --bench (RGB8 to the host), dragon 1080p (C3) and 4096^2.
# BANDS="1 2 4 8" sweeps ceres_render_f32's row bands (CERES_HOST_BANDS).  Outputs under gpurun_out/e2e/.
set -u; cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/${TAG:-e2e}; mkdir -p $OUT
A="data/dragon.obj --eye 0.0 -15.0 2.0 --dir 0.0 1.0 0.0 --up 0.0 0.0 1.0 --sun -50.0 -20.0 0.0 --rotate x 90.0"
for bands in ${BANDS:-4}; do
export CERES_HOST_BANDS=$bands
for sz in "1920 1080" "4096 4096"; do
  t=${sz/ /x}_b$bands
  timeout -k 10 120 tools/probes/dropin_bench $A --size $sz --reps ${REPS:-50} --out $OUT/dropin_$t.ppm > $OUT/dropin_$t.json 2> $OUT/dropin_$t.err || { cat $OUT/dropin_$t.err; exit 3; }
  echo "dropin $t $(cat $OUT/dropin_$t.json) sha=$(sha256sum $OUT/dropin_$t.ppm | cut -c1-64)"
  rm -f $OUT/dropin_$t.ppm
  timeout -k 10 120 ceres-raytracer_amd/render $A --fov 60 --size $sz --bench ${REPS:-50} --json -o $OUT/cli_$t.ppm > $OUT/cli_$t.log 2>&1 || { tail -3 $OUT/cli_$t.log; exit 3; }
  echo "cli $t $(tail -1 $OUT/cli_$t.log) sha=$(sha256sum $OUT/cli_$t.ppm | cut -c1-64)"
  rm -f $OUT/cli_$t.ppm
done
done
# C5=1: the 10M-triangle scene through the drop-in (3840x2160, host float framebuffer), with the
# per-call content hash (dropin_bench) and without it (dropin_bench_trust, CERES_DROPIN_TRUST_UNCHANGED)
if [ -n "${C5:-}" ]; then
  P="--proc 2237 --size 3840 2160 --eye 0.5 -0.4 0.6 --dir 0.0 0.9 -0.55 --up 0.0 0.0 1.0 --sun -50.0 -20.0 100.0"
  for b in dropin_bench dropin_bench_trust; do
    timeout -k 10 300 tools/probes/$b $P --reps ${C5_REPS:-10} --out $OUT/${b}_c5.ppm > $OUT/${b}_c5.json 2> $OUT/${b}_c5.err || { cat $OUT/${b}_c5.err; exit 3; }
    echo "$b c5 $(cat $OUT/${b}_c5.json) sha=$(sha256sum $OUT/${b}_c5.ppm | cut -c1-64)"
    rm -f $OUT/${b}_c5.ppm
  done
fi
