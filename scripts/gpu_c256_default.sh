# C = 256 trunk default switched to the 6-board one-buffer tiles (tower_wide.h): the tower tests and the
# full-size config-3 engine test on the new default, trunk-only timings (3-board / 6-board ring depth 2
# (default) / 6-board ring depth 4, SPMCTS_TOWER_CG=254; SKIP_TRUNK=1 skips them), then config 3 (plies
# 3-6) with the 6-board trunk (packed tails on 6-board tiles: the default), the 6-board trunk with
# 3-board tail code (SPMCTS_WIDE_TAILS=3) and the 3-board trunk, alternated.  Own time limit per step.
set -u
O=gpurun_out/c256d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_tower.py tests/test_gpu_engine.py -x -q -m gpu \
  -k "tower or config3 or wide or heads" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head; exit $rc; }
[ "${SKIP_TRUNK:-0}" = 1 ] || for rep in 1 2; do
  for v in 3 6 6d4; do
    c=${v:0:1}; cg=2; [ "$v" = 6d4 ] && cg=254
    SPMCTS_TOWER_C256=$c SPMCTS_TOWER_CG=$cg timeout -k 10 120 python3 scripts/bench_tower.py --trunk-only --ff 64 --batch 6144 --iters 10 > $O/one.json 2>$O/err.txt || { tail -3 $O/err.txt; exit 1; }
    echo "trunk C=256 6144 $v: $(python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), 'us', round(d['tflops'],1), 'TF/s')")" | tee -a $O/timing.txt
  done
done
for rep in 1 2; do
  for v in 6 6t3 3; do
    c=${v:0:1}; tl=6; [ "$v" = 6t3 ] && tl=3
    SPMCTS_TOWER_C256=$c SPMCTS_WIDE_TAILS=$tl timeout -k 10 400 python3 -u bench.py --games 16384 --sims 800 --filter-factor 64 --warmup 3 \
      --steps 4 --blocks-per-tree 2000 --no-cpu-baseline > $O/c3_$v.json 2> $O/c3_$v.err || { tail -5 $O/c3_$v.err; exit 1; }
    echo "config3 tiles $v: $(python3 -c "import json; d=json.loads([l for l in open('$O/c3_$v.json') if l.startswith('{')][0]); print(round(d['value'],1), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4))")" | tee -a $O/c3_tiles_ab.txt
  done
done
exit 0
