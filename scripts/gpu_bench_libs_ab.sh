# Bench A/B of library builds (LIBS="a.so b.so ..." under self_play_reinforcement_learning_amd/):
# trunk outputs of every build bit-equal to the first (scripts/tower_code_equal.py), then REPS rounds
# of the driver-form bench (warm-up 5, 20 plies), the builds alternated within each round.
set -u
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
L=$PWD/self_play_reinforcement_learning_amd
set -- $LIBS
FIRST=$1
SPMCTS_LIB=$L/$FIRST timeout -k 10 180 python3 scripts/tower_code_equal.py dump gpurun_out/ab/ref.npz || exit 1
for lib in "$@"; do
  [ "$lib" = "$FIRST" ] && continue
  SPMCTS_LIB=$L/$lib timeout -k 10 180 python3 scripts/tower_code_equal.py dump gpurun_out/ab/x.npz && \
  python3 scripts/tower_code_equal.py cmp gpurun_out/ab/ref.npz gpurun_out/ab/x.npz || exit 1
done
for rep in $(seq ${REPS:-3}); do
  for lib in "$@"; do
    SPMCTS_LIB=$L/$lib timeout -k 10 300 python3 bench.py --warmup ${W:-5} --steps ${S:-20} --no-cpu-baseline ${BARGS:-} > gpurun_out/ab/b.json 2>gpurun_out/ab/err.txt || { tail -3 gpurun_out/ab/err.txt; exit 1; }
    echo "bench w${W:-5} $lib: $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ab/b.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4))")" | tee -a gpurun_out/ab/summary.txt
  done
done
