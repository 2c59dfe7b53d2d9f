# rocprofv3 evidence for the bench: kernel-trace stats of the bench command, then separate
# PMC passes (FETCH_SIZE, WRITE_SIZE) restricted to the dominant kernel (k_tower*), reduced to
# per-launch traffic by scripts/pmc_traffic.py.
set -u
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
ARGS="--steps ${PSTEPS:-3} --warmup ${PWARM:-24} --no-cpu-baseline --lanes ${LANES:-2} --twin-no-dedup 0 --no-secondary ${EXTRA:-}"
# the timed region's dispatch count of a bench JSON line (the reducers keep only those)
ndisp() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(d[sys.argv[2]][sys.argv[3]])" "$@"; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof/trace -o run -- \
  python3 bench.py $ARGS > gpurun_out/prof/bench_traced.json 2> gpurun_out/prof/trace.err
rc=$?; echo "trace rc=$rc"; cut -c1-300 gpurun_out/prof/bench_traced.json
if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof/trace.err; exit $rc; fi
python3 scripts/tower_union.py gpurun_out/prof/trace/run_kernel_trace.csv ${LANES:-2} gpurun_out/prof/k_tower_union.json $(ndisp gpurun_out/prof/bench_traced.json roofline dispatches)
i=0
for set in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $set --kernel-include-regex "k_tower" -f csv -d gpurun_out/prof/pmc$i -o run -- \
     python3 bench.py $ARGS > gpurun_out/prof/pmc$i.json 2> gpurun_out/prof/pmc$i.err
  rc=$?; echo "pmc pass $i rc=$rc ($set)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/prof/pmc$i.err; exit $rc; fi
done
python3 scripts/pmc_traffic.py gpurun_out/prof/pmc1/run_counter_collection.csv \
  gpurun_out/prof/pmc2/run_counter_collection.csv gpurun_out/prof/k_tower_traffic.json ${LANES:-2} \
  $(ndisp gpurun_out/prof/pmc1.json roofline dispatches)
