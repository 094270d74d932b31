# GPU session: bench.py on every BASELINE.json config that fits one GPU (C1 bunny 640x480, C2 bunny 1080p
# primary-only, bunny 1080p full, C3 dragon 1080p, C4 dragon 4096^2, C5 10M triangles 4K),
# each with the reference CPU path timed beside it, then the weak-scaling rehearsal
# (tools/scaling_rehearsal.py).  Outputs under gpurun_out/${TAG:-sweep}/ (REHEARSE="" skips the rehearsal).
set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-sweep}
mkdir -p $OUT
step() { local t=$1; shift; local name=$1; shift; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; grep -v amdgpu.ids "$OUT/$name.log" | tail -1 | cut -c1-300; if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi; }
for c in ${CONFIGS:-bunny_640 bunny_1080_primary bunny_1080 dragon_1080 dragon_4096 proc_c5}; do
  steps=100; [ $c = proc_c5 ] && steps=20; [ $c = dragon_4096 ] && steps=50
  step 400 bench_$c python bench.py --config $c --steps $steps --warmup 5
done
for c in ${REHEARSE-dragon_1080 bunny_1080 dragon_4096}; do
  step 300 rehearsal_$c python tools/scaling_rehearsal.py $c 20 ${FPG:-8}
done
