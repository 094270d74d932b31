# bench.py at several --streams values (step k on stream k % S), repeated, C3 + C5.
set -u; cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/st; export TMPDIR=/tmp
run() { local n=$1; shift; timeout -k 10 300 "$@" > gpurun_out/st/$n.log 2>&1; local rc=$?; echo "$n rc=$rc $(grep -v amdgpu gpurun_out/st/$n.log | tail -1 | cut -c1-160)"; [ $rc -ne 0 ] && exit $rc; return 0; }
for rep in 1 2 3; do
  for S in ${SLIST:-1 2 4 8}; do run c3_s${S}_$rep python bench.py --steps 300 --warmup 10 --no-cpu-baseline --no-roofline --streams $S; done
done
for S in ${C5LIST:-1 4 8}; do run c5_s$S python bench.py --config proc_c5 --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --streams $S; done
