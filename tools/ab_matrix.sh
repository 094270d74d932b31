# A/B matrix: tools/ab.py over configs x step streams (16-frame batches of copies or orbit views)
# and solo frames, one GPU step per cell, each under its own time limit.
#   TAG=name  LIBS="a.so b.so"  CONFIGS="dragon_1080 ..."  STREAMS="1 8"  VIEW0="1 0"  SOLO="proc_c5 ..."
set -u; cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; OUT=gpurun_out/${TAG:-abm}; mkdir -p "$OUT"
for c in ${CONFIGS:-dragon_1080}; do
  for st in ${STREAMS:-1 8}; do
    for v in ${VIEW0:-1}; do
      f=$OUT/ab_${c}_s${st}_v$v.log
      AB_STREAMS=$st AB_FRAMES=16 AB_BATCH=16 AB_VIEW0=$v timeout -k 10 300 python tools/ab.py $c ${ROUNDS:-10} $LIBS > $f 2>&1 || { tail -3 $f; exit 1; }
      echo "$c streams=$st view0=$v $(tail -1 $f | cut -c1-600)"
    done
  done
done
for c in ${SOLO:-}; do
  f=$OUT/ab_${c}_solo.log
  timeout -k 10 300 python tools/ab.py $c ${ROUNDS_SOLO:-16} $LIBS > $f 2>&1 || { tail -3 $f; exit 1; }
  echo "$c solo $(tail -1 $f | cut -c1-600)"
done
exit 0
