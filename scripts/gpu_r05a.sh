# Round 5: the 16x16x32 C = 128 trunk with residue-parity B-fragment rows (tower_m16.h lane_row) against
# round 4's trunk (ab_libs/libspmcts_r04.so, built from the round-4 tree), one box:
# (1) bit-equality of the two libraries' outputs (scripts/tower_code_equal.py: 2- and 20-block nets, host and
#     device-count paths, fp16 and bf16); (2) the tower GPU tests on the new library; (3) LDS / stall PMC of
#     both trunks (trunk-only, 6,144 boards, fp16); (4) trunk-only timings alternated; (5) the driver-form bench
#     alternated (fp16, the bench default).
set -u
O=gpurun_out/r05a
mkdir -p $O
export TMPDIR=/tmp
NEW=$PWD/self_play_reinforcement_learning_amd/libspmcts.so
OLD=$PWD/ab_libs/libspmcts_r04.so
for dt in fp16 bf16; do
  for v in new old; do
    if [ $v = new ]; then LIB=$NEW; else LIB=$OLD; fi
    SPMCTS_LIB=$LIB timeout -k 10 180 python3 scripts/tower_code_equal.py dump $O/eq_${v}_$dt.npz 32 $dt > $O/eq.log 2>&1 || { tail -5 $O/eq.log; exit 1; }
  done
  python3 scripts/tower_code_equal.py cmp $O/eq_new_$dt.npz $O/eq_old_$dt.npz | tee -a $O/summary.txt
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_tower.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tower_tests.log 2>&1
rc=$?; tail -1 $O/tower_tests.log | tee -a $O/summary.txt; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/tower_tests.log | head -80; exit $rc; }
for v in new old; do
  if [ $v = new ]; then LIB=$NEW; else LIB=$OLD; fi
  SPMCTS_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-include-regex "k_tower" -f csv -d $O/p_$v -o run -- \
    python3 scripts/bench_tower.py --trunk-only --iters 10 --batch 6144 --dtype fp16 > $O/p.json 2> $O/p.err
  rc=$?; if [ $rc -ne 0 ]; then echo "pmc rc=$rc"; tail -5 $O/p.err; exit $rc; fi
  python3 scripts/tower_util.py $O/p_$v/run_counter_collection.csv $O/stall_$v.json
  rm -f $O/p_$v/run_counter_collection.csv
  echo "pmc $v: $(python3 -c "import json; d=json.load(open('$O/stall_$v.json')); print({k: round(v, 4) for k, v in d.items() if isinstance(v, float)})")" | tee -a $O/summary.txt
done
for BATCH in 1536 6144; do
  for dt in fp16 bf16; do
    for rep in 1 2; do
      for v in new old; do
        if [ $v = new ]; then LIB=$NEW; else LIB=$OLD; fi
        SPMCTS_LIB=$LIB timeout -k 10 120 python3 scripts/bench_tower.py --trunk-only --batch $BATCH --iters 20 --dtype $dt > $O/one.json 2>$O/err.txt || { tail -3 $O/err.txt; exit 1; }
        echo "trunk $BATCH $dt $v $(python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), round(d['tflops'],1))")" | tee -a $O/summary.txt
      done
    done
  done
done
for rep in 1 2; do
  for v in new old; do
    if [ $v = new ]; then LIB=$NEW; else LIB=$OLD; fi
    SPMCTS_LIB=$LIB timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline --twin-no-dedup 0 > $O/b_${v}_$rep.json 2>$O/err.txt || { tail -5 $O/err.txt; exit 1; }
    echo "bench $v: $(python3 -c "import json; d=json.loads([l for l in open('$O/b_${v}_$rep.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_us'],1), round(d['nn']['share_of_step'],4))")" | tee -a $O/summary.txt
  done
done
exit 0
