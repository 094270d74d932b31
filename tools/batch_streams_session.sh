# bench.py frames-per-step x streams grid at N = 1 (C3), repeated twice.
set -u; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/bs; export TMPDIR=/tmp
for rep in 1 2; do
for F in 1 2 4 8; do for S in 1 2 4 8; do
  timeout -k 10 120 python bench.py --frames $F --streams $S --steps $((400 / F)) --warmup 10 --no-cpu-baseline --no-roofline \
    > gpurun_out/bs/f${F}_s${S}_$rep.log 2>&1 || exit 1
  grep '^{' gpurun_out/bs/f${F}_s${S}_$rep.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('F=$F S=$S', d['value'], round(d['ms_per_step']/$F, 4))"
done; done; done
