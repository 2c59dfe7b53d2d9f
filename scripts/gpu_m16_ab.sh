# The 16x16x32 C = 128 trunk (tower_m16.h, the product default) against round 3's 32x32x16 set (the A/B
# library with SPMCTS_TOWER_M16=0), one box: (1) the tower GPU tests on the product library (fp32-reference
# tolerance, device- vs host-count paths, batch independence); (2) PMC clock / MFMA busy of both trunks
# (trunk-only, 6,144 boards, fp16); (3) trunk-only timings alternated, both dtypes; (4) the driver-form
# bench alternated (fp16, the bench default).
set -u
O=gpurun_out/m16
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/self_play_reinforcement_learning_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_tower.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tower_tests.log 2>&1
rc=$?; tail -1 $O/tower_tests.log | tee -a $O/summary.txt; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/tower_tests.log | head -80; exit $rc; }
for v in m16 old; do
  if [ $v = m16 ]; then E="SPMCTS_LIB=$L/libspmcts.so"; else E="SPMCTS_LIB=$L/libspmcts_ab.so SPMCTS_TOWER_M16=0"; fi
  env $E timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA --kernel-include-regex "k_tower" -f csv -d $O/p_$v -o run -- \
    python3 scripts/bench_tower.py --trunk-only --iters 10 --batch 6144 --dtype fp16 > $O/p.json 2> $O/p.err
  rc=$?; if [ $rc -ne 0 ]; then echo "pmc rc=$rc"; tail -5 $O/p.err; exit $rc; fi
  python3 scripts/tower_util.py $O/p_$v/run_counter_collection.csv $O/util_$v.json
  rm -f $O/p_$v/run_counter_collection.csv
  echo "pmc $v: $(python3 -c "import json; d=json.load(open('$O/util_$v.json')); print({k: round(v, 4) for k, v in d.items() if isinstance(v, float)})")" | tee -a $O/summary.txt
done
for BATCH in 1536 6144; do
  for dt in fp16 bf16; do
    for rep in 1 2; do
      for v in m16 old; do
        if [ $v = m16 ]; then E="SPMCTS_LIB=$L/libspmcts.so"; else E="SPMCTS_LIB=$L/libspmcts_ab.so SPMCTS_TOWER_M16=0"; fi
        env $E timeout -k 10 120 python3 scripts/bench_tower.py --trunk-only --batch $BATCH --iters 20 --dtype $dt > $O/one.json 2>$O/err.txt || { tail -3 $O/err.txt; exit 1; }
        echo "trunk $BATCH $dt $v $(python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), round(d['tflops'],1))")" | tee -a $O/summary.txt
      done
    done
  done
done
for rep in 1 2; do
  for v in m16 old; do
    if [ $v = m16 ]; then E="SPMCTS_LIB=$L/libspmcts.so"; else E="SPMCTS_LIB=$L/libspmcts_ab.so SPMCTS_TOWER_M16=0"; fi
    env $E timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline --twin-no-dedup 0 > $O/b_${v}_$rep.json 2>$O/err.txt || { tail -5 $O/err.txt; exit 1; }
    echo "bench $v: $(python3 -c "import json; d=json.loads([l for l in open('$O/b_${v}_$rep.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_us'],1), round(d['nn']['share_of_step'],4))")" | tee -a $O/summary.txt
  done
done
exit 0
