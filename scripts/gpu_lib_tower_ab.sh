# Two library builds (LIBS="prev.so new.so"): trunk outputs bit-equal (scripts/tower_code_equal.py),
# tower GPU tests on the new build, trunk-only timings at one and four rounds, bench A/B (short run).
set -u
mkdir -p gpurun_out/lt
export TMPDIR=/tmp
L=$PWD/self_play_reinforcement_learning_amd
set -- $LIBS
A=$1; B=$2
SPMCTS_LIB=$L/$A timeout -k 10 180 python3 scripts/tower_code_equal.py dump gpurun_out/lt/a.npz && \
SPMCTS_LIB=$L/$B timeout -k 10 180 python3 scripts/tower_code_equal.py dump gpurun_out/lt/b.npz || exit 1
# NOEQ=1: a numerics change (the tower tests below are then the check); the comparison is printed
python3 scripts/tower_code_equal.py cmp gpurun_out/lt/a.npz gpurun_out/lt/b.npz || [ "${NOEQ:-0}" = 1 ] || exit 1
SPMCTS_LIB=$L/$B timeout -k 10 300 python -u -m pytest tests/test_gpu_tower.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/lt/tests.log 2>&1
rc=$?; tail -1 gpurun_out/lt/tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for BATCH in 1536 6144; do
  for rep in 1 2; do
    for lib in $A $B; do
      SPMCTS_LIB=$L/$lib timeout -k 10 120 python3 scripts/bench_tower.py --trunk-only --batch $BATCH --iters 20 > gpurun_out/lt/one.json 2>gpurun_out/lt/err.txt || { tail -3 gpurun_out/lt/err.txt; exit 1; }
      echo "trunk $BATCH $lib $(python3 -c "import json; d=json.loads(open('gpurun_out/lt/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), round(d['tflops'],1))")"
    done
  done
done
for rep in 1 2; do
  for lib in $A $B; do
    SPMCTS_LIB=$L/$lib timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/lt/b.json 2>gpurun_out/lt/err.txt || { tail -3 gpurun_out/lt/err.txt; exit 1; }
    echo "bench w5 $lib: $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/lt/b.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4))")"
  done
done
