# C = 256 residual scratch through a buffer resource (A/B library, SPMCTS_TOWER_CG 2561 = nt cache policy as
# the pointer form's nontemporal accesses, 2562 = default policy) against the product library's pointer form:
# trunk outputs of the 2- and 20-block ResNet-256 compared bit for bit (scripts/tower_code_equal.py, host path),
# then trunk-only timings (6,144 boards) of each, alternated.
set -u
mkdir -p gpurun_out/rsrc
export TMPDIR=/tmp
L=$PWD/self_play_reinforcement_learning_amd
SPMCTS_LIB=$L/libspmcts.so timeout -k 10 240 python3 scripts/tower_code_equal.py dump gpurun_out/rsrc/ref.npz 64 || exit 1
for code in 2561 2562; do
  SPMCTS_LIB=$L/libspmcts_ab.so SPMCTS_TOWER_CG=$code timeout -k 10 240 python3 scripts/tower_code_equal.py dump gpurun_out/rsrc/x$code.npz 64 || exit 1
  echo "code $code: $(python3 scripts/tower_code_equal.py cmp gpurun_out/rsrc/ref.npz gpurun_out/rsrc/x$code.npz)" | tee -a gpurun_out/rsrc/summary.txt
done
for rep in 1 2; do
  for code in none 2561 2562; do
    if [ $code = none ]; then lib=libspmcts.so; env=""; else lib=libspmcts_ab.so; env="SPMCTS_TOWER_CG=$code"; fi
    env SPMCTS_LIB=$L/$lib $env timeout -k 10 120 python3 scripts/bench_tower.py --trunk-only --ff 64 --batch 6144 --iters 10 > gpurun_out/rsrc/one.json 2>gpurun_out/rsrc/err.txt || { tail -3 gpurun_out/rsrc/err.txt; exit 1; }
    echo "trunk C256 6144 $code $(python3 -c "import json; d=json.loads(open('gpurun_out/rsrc/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), round(d['tflops'],1))")" | tee -a gpurun_out/rsrc/summary.txt
  done
done
