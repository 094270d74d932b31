# DRAM writes of a 16-frame batch launch against the batch kernel's VGPR budget: rocprofv3 --pmc
# WRITE_SIZE of tools/batch_launch.py per build (the in-tree library and $LIBS, CERES_LIB), then the
# same builds' throughput through tools/ab_matrix.sh.  One PMC pass per run, each under its own limit.
#   TAG=name  LIBS="ceres-raytracer_amd/variants/libceres_hip_x.so"  CONFIGS="dragon_1080 bunny_1080"
set -u; cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/${TAG:-spill}; mkdir -p "$OUT"
for c in ${CONFIGS:-dragon_1080 bunny_1080}; do
  for lib in ceres-raytracer_amd/libceres_hip.so ${LIBS:-}; do
    v=$(basename $lib .so)
    CERES_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_WR --output-format csv \
      -d $OUT/pmc_${c}_$v -o run -- python3 tools/batch_launch.py $c fma 16 5 > $OUT/pmc_${c}_$v.log 2>&1 || { echo "FAIL pmc $c $v"; exit 1; }
    python3 - $OUT/pmc_${c}_$v <<'PY' || exit 3
import csv, glob, sys, collections
rows = [r for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in rows:
    if "ceres_fused" not in r["Kernel_Name"]: continue
    acc[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
    n[(r["Kernel_Name"][:60], r["Counter_Name"])] += 1
for k, d in acc.items():
    print(sys.argv[1].split("/")[-1], k, {c: round(v / n[(k, c)], 1) for c, v in d.items()})
PY
  done
done
LIBS="ceres-raytracer_amd/libceres_hip.so ${LIBS:-}" TAG=${TAG:-spill}/ab CONFIGS="${CONFIGS:-dragon_1080 bunny_1080}" STREAMS=8 ROUNDS=${ROUNDS:-10} SOLO="${SOLO:-}" bash tools/ab_matrix.sh
