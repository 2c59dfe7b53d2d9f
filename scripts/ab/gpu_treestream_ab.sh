# Same-box A/B: tree kernels + heads on a high-priority stream per lane (SPMCTS_TREE_STREAM=1) vs one stream.
set -u
mkdir -p gpurun_out/ts
export TMPDIR=/tmp
SPMCTS_TREE_STREAM=1 timeout -k 10 300 python -m pytest tests/test_gpu_engine.py -x -q -m gpu -k "laned or full_size_headline" --timeout 200 --timeout-method thread > gpurun_out/ts/tests.log 2>&1
rc=$?; tail -1 gpurun_out/ts/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for W in "5 20" "24 40"; do
  set -- $W
  for E in 0 1 0 1; do
    SPMCTS_TREE_STREAM=$E timeout -k 10 300 python3 bench.py --warmup $1 --steps $2 --no-cpu-baseline > gpurun_out/ts/b.json 2> gpurun_out/ts/err.txt || { tail -3 gpurun_out/ts/err.txt; exit 1; }
    echo "warmup $1 tree_stream $E: $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ts/b.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4))")"
  done
done
