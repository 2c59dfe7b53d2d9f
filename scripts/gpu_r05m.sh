# Round 5: the C = 256 trunk on 16x16x32 one-buffer tiles (tower_wide16.h, the product default) -- GPU tower
# tests, trunk-only timing against round 4's 32x32x16 tiles (A/B library SPMCTS_TOWER_C256=32) alternated,
# then config 3 near steady state (32 warm-up plies, 6 timed, two lanes) with each.
set -u
O=gpurun_out/r05m
mkdir -p $O
export TMPDIR=/tmp
AB=$PWD/self_play_reinforcement_learning_amd/libspmcts_ab.so
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_tower.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
for rep in 1 2 3; do
  for v in wide16 wide32; do
    if [ $v = wide16 ]; then E=""; else E="SPMCTS_LIB=$AB SPMCTS_TOWER_C256=32"; fi
    env $E timeout -k 10 180 python3 scripts/bench_tower.py --trunk-only --batch 6144 --ff 64 --iters 10 > $O/one.json 2>$O/err.txt || { tail -3 $O/err.txt; exit 1; }
    echo "c256 trunk 6144 $v: $(python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), 'us', round(d['tflops'],1), 'TF/s')")" | tee -a $O/summary.txt
  done
done
for v in wide16 wide32; do
  if [ $v = wide16 ]; then E=""; else E="SPMCTS_LIB=$AB SPMCTS_TOWER_C256=32"; fi
  env $E timeout -k 10 540 python3 -u bench.py --games 16384 --sims 800 --filter-factor 64 --warmup 32 --steps 6 \
    --blocks-per-tree 8000 --twin-no-dedup 0 --no-cpu-baseline --progress --lanes 2 \
    > $O/c3_$v.json 2> $O/c3_$v.err || { tail -3 $O/c3_$v.err; exit 1; }
  echo "config3 $v: $(python3 -c "import json; d=json.loads([l for l in open('$O/c3_$v.json') if l.startswith('{')][0]); print(round(d['value'],1), round(d['roofline']['frac'],4), d['nn']['rows_per_leaf'], round(d['nn']['share_of_step'],4))")" | tee -a $O/summary.txt
done
exit 0
