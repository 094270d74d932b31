# PMC passes (one counter group per rocprofv3 run, never combined with tracing) on a short
# render loop.  usage: GROUPS="A B;C D" CMD="python3 tools/ab.py dragon_1080 5 wave" bash tools/pmc_session.sh
set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/pmc; mkdir -p $OUT
CMD=${CMD:-python3 tools/ab.py dragon_1080 5 wave}
i=0
IFS=';' read -ra GRPS <<< "${GROUPS_PMC}"
for g in "${GRPS[@]}"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $g --output-format csv -d $OUT/p$i -o run -- $CMD > $OUT/p$i.log 2>&1; rc=$?
  echo "pass $i ($g) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
python3 tools/pmc_summary.py ${PMC_CFG:-dragon_1080_diag} $OUT $OUT/summary.json > /dev/null && cat $OUT/summary.json
