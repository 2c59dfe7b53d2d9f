# One tree per wave (SPMCTS_TREE_BLOCK=8) vs 8 trees per wave (64): threaded parity, isolated tree
# kernels, and same-box steady-state bench A/B.
set -u
mkdir -p gpurun_out/tb
export TMPDIR=/tmp
SPMCTS_TREE_BLOCK=8 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k threaded --timeout 120 --timeout-method thread > gpurun_out/tb/parity8.log 2>&1
rc=$?; tail -1 gpurun_out/tb/parity8.log; if [ $rc -ne 0 ]; then exit $rc; fi
for B in 64 8 64 8; do
  SPMCTS_TREE_BLOCK=$B timeout -k 10 120 python3 scripts/bench_tree.py > gpurun_out/tb/iso_$B.json 2>/dev/null || exit 1
  echo "iso block $B: $(cat gpurun_out/tb/iso_$B.json | cut -c1-260)"
done
for B in 64 8 64 8; do
  SPMCTS_TREE_BLOCK=$B timeout -k 10 300 python3 bench.py --warmup 24 --steps 40 --no-cpu-baseline > gpurun_out/tb/b_$B.json 2>gpurun_out/tb/err.txt || { tail -3 gpurun_out/tb/err.txt; exit 1; }
  echo "bench block $B: $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/tb/b_$B.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4), round(d['tree_roofline']['expand']['ms']/max(1,d['tree_roofline']['expand']['dispatches'])*1e3,1))")"
done
