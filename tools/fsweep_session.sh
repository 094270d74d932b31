set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/fsweep
for f in 8 16 32 64 16; do
  timeout -k 10 300 python bench.py --frames-per-gpu $f --steps 100 --warmup 10 --no-cpu-baseline --no-roofline > gpurun_out/fsweep/f$f.log 2>&1 || { echo "fail $f"; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('gpurun_out/fsweep/f$f.log') if l.startswith('{')][-1]); print($f, d['value'], d['ms_per_step'])"
done
