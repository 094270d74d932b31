# Build libceres_hip_<tag>.so from git revision <rev> (whole library, via a temporary worktree)
# for tools/ab.py A/B runs.
# usage: bash tools/build_rev_variant.sh <rev> <tag> [extra hipcc defs]
set -eu
rev=$1; tag=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" worktree add --detach "$tmp/wt" "$rev" > /dev/null
trap 'git -C "$root" worktree remove --force "$tmp/wt"; rm -rf "$tmp"' EXIT
make -C "$tmp/wt/ceres-raytracer_amd/csrc" -j8 "$tmp/wt/ceres-raytracer_amd/libceres_hip.so" \
     HIPFLAGS_EXTRA="$*" > "$tmp/build.log" 2>&1 || { tail -20 "$tmp/build.log"; exit 1; }
mkdir -p "$root/ceres-raytracer_amd/variants"
cp "$tmp/wt/ceres-raytracer_amd/libceres_hip.so" "$root/ceres-raytracer_amd/variants/libceres_hip_$tag.so"
echo "built variants/libceres_hip_$tag.so from $rev"
