# Build libceres_hip_<tag>.so from the csrc of git revision <rev> (for tools/ab.py A/B runs).
# usage: bash tools/build_rev_variant.sh <rev> <tag> [extra hipcc defs]
set -eu
rev=$1; tag=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
for f in render_hip.hip scene_host.cpp ceres_types.hpp host_common.hpp pow24.hpp; do
  git -C "$root" show "$rev:ceres-raytracer_amd/csrc/$f" > "$tmp/$f"
done
git -C "$root" show "$rev:include/ceres_render.h" > "$tmp/ceres_render.h"
mkdir -p "$root/ceres-raytracer_amd/variants"
H="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -munsafe-fp-atomics -I$tmp"
/opt/rocm/bin/hipcc $H "$@" -c "$tmp/render_hip.hip" -o "$tmp/r.o"
g++ -O3 -std=c++17 -fPIC -ffp-contract=off -mavx2 -mfma -fopenmp -I$tmp -D__HIP_PLATFORM_AMD__ -c "$tmp/scene_host.cpp" -o "$tmp/s.o"
g++ -shared -o "$root/ceres-raytracer_amd/variants/libceres_hip_$tag.so" "$tmp/r.o" "$tmp/s.o" -L/opt/rocm/lib -lamdhip64 -fopenmp -Wl,-rpath,/opt/rocm/lib
rm -rf "$tmp"
echo "built variants/libceres_hip_$tag.so from $rev"
