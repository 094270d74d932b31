# One-GPU multi-GPU rehearsal (tools/scaling_rehearsal.py) per setting of $VAR over $VALS, for $CFGS.
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06w}; mkdir -p "$OUT"
for c in ${CFGS:-dragon_1080}; do
  for v in ${VALS:-0}; do
    env ${VAR:-CERES_ASSEMBLE_ROWS}=$v timeout -k 10 400 python tools/scaling_rehearsal.py $c ${REPS:-10} 16 ${RB:-16} > $OUT/rehearsal_${c}_$(basename $v).json 2> $OUT/rehearsal_${c}_$(basename $v).err || { echo "FAIL $c $v"; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/rehearsal_${c}_$(basename $v).json'))['by_n']['8']
print('$c', '$v', 'render', d['predicted_weak_efficiency_pipelined'], 'exchange', d['predicted_weak_efficiency_pipelined_with_exchange'], 'bands', d.get('predicted_weak_efficiency_bands'), d.get('predicted_weak_efficiency_bands_with_exchange'))"
  done
done
