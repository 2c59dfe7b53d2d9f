# Round 5: variants of the 16x16x32 one-buffer C = 256 trunk (A/B library): the product form (2560), a 4-deep
# weight ring (2564), the compiler's own k-loop schedule (2556); trunk-only 6,144 boards bf16, alternated.
set -u
O=gpurun_out/r05aa
mkdir -p $O
export TMPDIR=/tmp
AB=$PWD/self_play_reinforcement_learning_amd/libspmcts_ab.so
for rep in 1 2 3; do
  for c in 2560 2564 2556; do
    SPMCTS_LIB=$AB SPMCTS_TOWER_CG=$c timeout -k 10 180 python3 scripts/bench_tower.py --trunk-only --batch 6144 --ff 64 --iters 10 > $O/one.json 2>$O/err.txt || { tail -3 $O/err.txt; exit 1; }
    echo "c256 trunk 6144 code $c: $(python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), 'us', round(d['tflops'],1), 'TF/s')")" | tee -a $O/summary.txt
  done
done
exit 0
