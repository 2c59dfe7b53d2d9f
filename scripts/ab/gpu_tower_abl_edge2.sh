# Edge-tile trunk: weight-stream ablations (16 = no weight loads, 128 = half the weight bytes) and ring
# depth 8 (case 250) against the shipped depth 4, at one round (1,536 boards) and four (6,144).
set -u
mkdir -p gpurun_out/abl2
export TMPDIR=/tmp
: > gpurun_out/abl2/abl.txt
for B in 1536 6144; do
  for rep in 1 2; do
    for C in ${CGS:-200 216 328 250}; do
      SPMCTS_TOWER_CG=$C timeout -k 10 120 python3 scripts/bench_tower.py --trunk-only --batch $B --iters 20 > gpurun_out/abl2/one.json 2> gpurun_out/abl2/err.txt || { tail -3 gpurun_out/abl2/err.txt; exit 1; }
      echo "batch $B cg $C $(python3 -c "import json; d=json.loads(open('gpurun_out/abl2/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), round(d.get('tflops',0),1))")" | tee -a gpurun_out/abl2/abl.txt
    done
  done
done
