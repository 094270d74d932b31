set -u
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out/r06v
for rep in 1 2; do
for cfg in "16 8" "32 8" "24 8" "16 4" "32 4" "48 8" "16 12"; do
  set -- $cfg
  timeout -k 10 200 python bench.py --frames-per-gpu $1 --streams $2 --steps 40 --warmup 10 --no-roofline --no-cpu-baseline --no-orbit --no-alt --no-count > gpurun_out/r06v/fpg$1_s$2_r$rep.log 2>&1 || { echo "FAIL $cfg"; exit 1; }
  python3 -c "import json,sys; l=[x for x in open('gpurun_out/r06v/fpg$1_s$2_r$rep.log') if x.startswith('{')][-1]; d=json.loads(l); print('$1 $2 r$rep', d['value'], d['ms_per_step'])"
done
done
