# rocprofv3 evidence for the tree kernels (k_select_vl + k_expand_vl) on the default bench command:
# kernel-trace stats, then separate FETCH_SIZE / WRITE_SIZE passes restricted to the tree kernels.
set -u
mkdir -p gpurun_out/tree
export TMPDIR=/tmp
ARGS="--steps ${PSTEPS:-3} --warmup ${PWARM:-24} --no-cpu-baseline --twin-no-dedup 0 --no-secondary ${EXTRA:-}"
ndisp() { python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(d[sys.argv[2]][sys.argv[3]])" "$@"; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/tree/trace -o run -- \
  python3 bench.py $ARGS > gpurun_out/tree/bench_traced.json 2> gpurun_out/tree/trace.err
rc=$?; echo "trace rc=$rc"
if [ $rc -ne 0 ]; then tail -5 gpurun_out/tree/trace.err; exit $rc; fi
i=0
for set in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $set --kernel-include-regex "k_select_vl|k_expand_vl" -f csv \
     -d gpurun_out/tree/pmc$i -o run -- python3 bench.py $ARGS > gpurun_out/tree/pmc$i.json 2> gpurun_out/tree/pmc$i.err
  rc=$?; echo "pmc pass $i rc=$rc ($set)"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/tree/pmc$i.err; exit $rc; fi
done
python3 scripts/pmc_tree.py gpurun_out/tree/pmc1/run_counter_collection.csv \
  gpurun_out/tree/pmc2/run_counter_collection.csv gpurun_out/tree/tree_traffic.json \
  $(ndisp gpurun_out/tree/pmc1.json tree_roofline launches)
