# GPU session: Morton lane order in the f64 kernel (CERES_LANE_QUADS64), A/B through the CLI
# (./render --double --bench) alternating the default build and ceres-raytracer_amd/variants/q64,
# output PPMs compared byte for byte.
set -u; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2 3 4; do
  for v in ceres-raytracer_amd ceres-raytracer_amd/variants/q64; do
    t=$(basename $v)
    timeout -k 10 120 $v/render data/dragon.obj --rotate x 90 --double --bench 30 --json -o /tmp/d_$t.ppm > gpurun_out/q64_$t.log 2>&1 || { tail -5 gpurun_out/q64_$t.log; exit 3; }
    echo "dragon $t $(tail -1 gpurun_out/q64_$t.log | cut -c1-300)"
    timeout -k 10 120 $v/render data/bunny.obj --eye 0 .1 -.3 --dir 0 0 1 --up 0 1 0 --rotate y -145 --size 1920 1080 --double --bench 30 --json -o /tmp/b_$t.ppm > gpurun_out/q64b_$t.log 2>&1 || { tail -5 gpurun_out/q64b_$t.log; exit 3; }
    echo "bunny $t $(tail -1 gpurun_out/q64b_$t.log | cut -c1-300)"
  done
done
cmp /tmp/d_ceres-raytracer_amd.ppm /tmp/d_q64.ppm && cmp /tmp/b_ceres-raytracer_amd.ppm /tmp/b_q64.ppm && echo "ppm identical"
