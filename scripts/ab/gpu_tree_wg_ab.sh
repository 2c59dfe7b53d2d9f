# Tree-kernel workgroup size (SPMCTS_TREE_BLOCK = 64 / 256 / 512 threads): threaded parity at 512, isolated
# tree kernels, and same-box bench A/B in the driver's short form and in steady state.
set -u
mkdir -p gpurun_out/twg
export TMPDIR=/tmp
SPMCTS_TREE_BLOCK=512 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_engine.py -x -q -m gpu -k "threaded or vl or K4 or search_threads" --timeout 200 --timeout-method thread > gpurun_out/twg/parity512.log 2>&1
rc=$?; tail -1 gpurun_out/twg/parity512.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" gpurun_out/twg/parity512.log | head; exit $rc; fi
for B in 64 512 64 512; do
  SPMCTS_TREE_BLOCK=$B timeout -k 10 120 python3 scripts/bench_tree.py > gpurun_out/twg/iso.json 2>/dev/null || exit 1
  echo "iso block $B: $(python3 -c "import json; d=json.loads(open('gpurun_out/twg/iso.json').read().strip().splitlines()[-1]); print(round(d['select_avg_us'],1), round(d['expand_avg_us'],1))")"
done
for W in "5 20" "24 40"; do
  set -- $W
  for B in ${BLOCKS:-64 512 256 64 512 256}; do
    SPMCTS_TREE_BLOCK=$B timeout -k 10 300 python3 bench.py --warmup $1 --steps $2 --no-cpu-baseline > gpurun_out/twg/b.json 2>gpurun_out/twg/err.txt || { tail -3 gpurun_out/twg/err.txt; exit 1; }
    echo "bench w$1 block $B: $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/twg/b.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4), round(d['tree_roofline']['expand']['ms']/max(1,d['tree_roofline']['expand']['dispatches'])*1e3,1))")"
  done
done
