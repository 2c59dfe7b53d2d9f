# Round 5: the C = 256 trunk with one layer-loop iteration per residual block (no odd/even branch) and tap 0's
# rows read from the LDS table per layer (spills 66 -> 20), and every device-count tile a 6-board tile, against
# round 4's library (ab_libs/libspmcts_r04.so), one box: (1) bit-equality of the outputs (ResNet-256, 2 and 20
# blocks, host and device-count paths, fp16 and bf16); (2) the C = 256 tile test (6-board vs 3-board tiles);
# (3) config 3 (16,384 games, 800 sims, ResNet-256x20), plies 3-6, alternated; (4) the config-5 arena test.
set -u
O=gpurun_out/r05b
mkdir -p $O
export TMPDIR=/tmp
NEW=$PWD/self_play_reinforcement_learning_amd/libspmcts.so
OLD=$PWD/ab_libs/libspmcts_r04.so
for dt in fp16 bf16; do
  for v in new old; do
    if [ $v = new ]; then LIB=$NEW; else LIB=$OLD; fi
    SPMCTS_LIB=$LIB timeout -k 10 240 python3 scripts/tower_code_equal.py dump $O/eq_${v}_$dt.npz 64 $dt > $O/eq.log 2>&1 || { tail -5 $O/eq.log; exit 1; }
  done
  python3 scripts/tower_code_equal.py cmp $O/eq_new_$dt.npz $O/eq_old_$dt.npz | tee -a $O/summary.txt
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_tower.py -m gpu -x -q --timeout 300 --timeout-method thread -k "wide_c256 or c256 or 256" > $O/tower_tests.log 2>&1
rc=$?; tail -1 $O/tower_tests.log | tee -a $O/summary.txt; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/tower_tests.log | head -80; exit $rc; }
for rep in 1 2; do
  for v in new old; do
    if [ $v = new ]; then LIB=$NEW; else LIB=$OLD; fi
    SPMCTS_LIB=$LIB timeout -k 10 240 python3 -u bench.py --games 16384 --sims 800 --filter-factor 64 --warmup 2 --steps 4 \
      --blocks-per-tree 8000 --twin-no-dedup 0 --no-cpu-baseline > $O/c3_${v}_$rep.json 2>$O/err.txt || { tail -5 $O/err.txt; exit 1; }
    echo "config3 plies 3-6 $v: $(python3 -c "import json; d=json.loads([l for l in open('$O/c3_${v}_$rep.json') if l.startswith('{')][0]); print(round(d['value'],1), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_us'],1))")" | tee -a $O/summary.txt
  done
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -m gpu -x -v -s --timeout 360 --timeout-method thread -k "config5" > $O/config5_test.log 2>&1
rc=$?; grep -E "config5:|passed|failed" $O/config5_test.log | tee -a $O/summary.txt; [ $rc -eq 0 ] || { tail -40 $O/config5_test.log; exit $rc; }
exit 0
