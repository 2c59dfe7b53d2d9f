# Timing ablations of the shipped edge-tile trunk (results wrong by design; SPMCTS_TOWER_CG=200+X):
# 2 = no epilogue, 4 = no inter-layer barrier, 8 = no LDS operand reads, 16 = no weight loads.
# One full round (1,536 boards = 256 workgroups of 6), trunk only.
set -u
mkdir -p gpurun_out/abl
export TMPDIR=/tmp
: > gpurun_out/abl/abl.txt
for rep in 1 2; do
  for X in 0 2 4 6 8 16 24 30; do
    SPMCTS_TOWER_CG=$((200 + X)) timeout -k 10 120 python3 scripts/bench_tower.py --trunk-only --batch ${BATCH:-1536} --iters 20 > gpurun_out/abl/one.json 2> gpurun_out/abl/err.txt || { tail -3 gpurun_out/abl/err.txt; exit 1; }
    echo "abl $X $(python3 -c "import json; d=json.loads(open('gpurun_out/abl/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), round(d.get('tflops',0),1))")" | tee -a gpurun_out/abl/abl.txt
  done
done
