# Diagnostics: fused-kernel wave timeline + tail/throughput probe (outputs under gpurun_out/diag/).
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/diag; mkdir -p $OUT
step() { local t=$1; shift; local name=$1; shift; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log"; echo "STOP after $name"; exit $rc; fi; }
for c in ${CONFIGS:-dragon_1080}; do
  step 300 timeline_$c python tools/fused_timeline.py $c
  step 300 tail_$c python tools/tail_diag.py $c
done
