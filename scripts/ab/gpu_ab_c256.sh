# Trunk-only A/B of two library builds at C = 256 (config 3) and C = 128 (control): session-start build vs HEAD.
set -u
mkdir -p gpurun_out/ab256
L=$PWD/self_play_reinforcement_learning_amd
for rep in 1 2; do
for cfg in "64 4096" "64 16384" "32 6144"; do
  set -- $cfg
  for lib in libspmcts_old.so libspmcts.so; do
    SPMCTS_LIB=$L/$lib timeout -k 10 120 python3 scripts/bench_tower.py --trunk-only --ff $1 --batch $2 --iters 10 > gpurun_out/ab256/one.json 2>gpurun_out/ab256/err.txt || { tail -3 gpurun_out/ab256/err.txt; exit 1; }
    echo "ff $1 batch $2 $lib $(python3 -c "import json; d=json.loads(open('gpurun_out/ab256/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), round(d['tflops'],1))")" | tee -a gpurun_out/ab256/summary.txt
  done
done
done
