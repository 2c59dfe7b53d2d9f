set -u
mkdir -p gpurun_out/iso
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in ${LIBS}; do
    SPMCTS_LIB=$PWD/self_play_reinforcement_learning_amd/$lib timeout -k 10 120 python3 scripts/bench_tree.py > gpurun_out/iso/iso.json 2>gpurun_out/iso/err.txt || { tail -3 gpurun_out/iso/err.txt; exit 1; }
    echo "iso $lib: $(python3 -c "import json; d=json.loads(open('gpurun_out/iso/iso.json').read().strip().splitlines()[-1]); print(round(d['select_avg_us'],1), round(d['expand_avg_us'],1))")"
  done
done
