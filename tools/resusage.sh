# Kernel resource usage (VGPRs, SGPRs, scratch, spills, occupancy) of render_hip.hip's fused
# kernels for a set of -D defines:  bash tools/resusage.sh "-DCERES_PK_SLAB=0"
set -e
cd "$(dirname "$0")/../ceres-raytracer_amd/csrc"
out=$(mktemp)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-slp-vectorize -fhip-fp32-correctly-rounded-divide-sqrt \
  -fno-gpu-flush-denormals-to-zero -munsafe-fp-atomics -I../../include $1 \
  --cuda-device-only -c -Rpass-analysis=kernel-resource-usage -o /dev/null render_hip.hip 2> "$out" || true
python3 - "$out" <<'PY'
import re, sys
t = open(sys.argv[1]).read()
for blk in t.split("Function Name: ")[1:]:
    name = blk.split()[0]
    if "fused" not in name: continue
    g = lambda k: (re.search(k + r": (\d+)", blk) or [0, 0])[1]
    print(name[22:90], "V", g("VGPRs"), "S", g("TotalSGPRs"), "scr", g(r"ScratchSize \[bytes/lane\]"),
          "sspill", g("SGPRs Spill"), "vspill", g("VGPRs Spill"), "occ", g(r"Occupancy \[waves/SIMD\]"))
PY
rm -f "$out"
