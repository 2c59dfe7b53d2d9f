# C = 256 trunk A/B of library builds (LIBS="a.so b.so" under self_play_reinforcement_learning_amd/, the first
# is the reference): outputs of every build bit-equal to the first's (scripts/tower_code_equal.py at
# ResNet-256, host and device-count paths), then trunk-only timings at 6,144 boards and config 3 (plies
# 3-6), the builds alternated.  Own time limit per step.
set -u -o pipefail
O=gpurun_out/c256libs
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/self_play_reinforcement_learning_amd
set -- $LIBS
FIRST=$1
SPMCTS_LIB=$L/$FIRST timeout -k 10 300 python3 scripts/tower_code_equal.py dump $O/ref.npz 64 || exit 1
for lib in "$@"; do
  [ "$lib" = "$FIRST" ] && continue
  SPMCTS_LIB=$L/$lib timeout -k 10 300 python3 scripts/tower_code_equal.py dump $O/x.npz 64 && \
  python3 scripts/tower_code_equal.py cmp $O/ref.npz $O/x.npz | tee -a $O/summary.txt || exit 1
done
for rep in ${REPS:-1 2}; do
  for lib in "$@"; do
    SPMCTS_LIB=$L/$lib timeout -k 10 120 python3 scripts/bench_tower.py --trunk-only --ff 64 --batch 6144 --iters 10 > $O/one.json 2>$O/err.txt || { tail -3 $O/err.txt; exit 1; }
    echo "trunk C=256 6144 $lib: $(python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), 'us', round(d['tflops'],1), 'TF/s')")" | tee -a $O/summary.txt
  done
done
for rep in ${REPS:-1 2}; do
  for lib in "$@"; do
    SPMCTS_LIB=$L/$lib timeout -k 10 400 python3 -u bench.py --games 16384 --sims 800 --filter-factor 64 --warmup 3 \
      --steps 4 --blocks-per-tree 2000 --no-cpu-baseline > $O/c3.json 2> $O/c3.err || { tail -5 $O/c3.err; exit 1; }
    echo "config3 $lib: $(python3 -c "import json; d=json.loads([l for l in open('$O/c3.json') if l.startswith('{')][0]); print(round(d['value'],1), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4))")" | tee -a $O/summary.txt
  done
done
exit 0
