# Group-shared Philox jitter: games identical to the previous build (Philox mode), parity/statistical
# GPU tests, isolated tree kernels and bench A/B against the previous build.
set -u
mkdir -p gpurun_out/rg
export TMPDIR=/tmp
L=$PWD/self_play_reinforcement_learning_amd
SPMCTS_LIB=$L/libspmcts_prev.so timeout -k 10 200 python3 scripts/rng_equal.py gpurun_out/rg/prev.npz > gpurun_out/rg/eq.log 2>&1 || { tail -5 gpurun_out/rg/eq.log; exit 1; }
SPMCTS_LIB=$L/libspmcts.so timeout -k 10 200 python3 scripts/rng_equal.py gpurun_out/rg/new.npz >> gpurun_out/rg/eq.log 2>&1 || { tail -5 gpurun_out/rg/eq.log; exit 1; }
python3 scripts/rng_equal.py --compare gpurun_out/rg/prev.npz gpurun_out/rg/new.npz || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_statistical.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/rg/tests.log 2>&1
rc=$?; tail -1 gpurun_out/rg/tests.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" gpurun_out/rg/tests.log | head; exit $rc; fi
LIBS="libspmcts_prev.so libspmcts.so" bash scripts/gpu_iso_ab.sh
for rep in 1 2; do
  for lib in libspmcts_prev.so libspmcts.so; do
    SPMCTS_LIB=$L/$lib timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline > gpurun_out/rg/b.json 2>gpurun_out/rg/err.txt || { tail -3 gpurun_out/rg/err.txt; exit 1; }
    echo "bench w5 $lib: $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/rg/b.json') if l.startswith('{')][0]); print(round(d['value']), round(d['nn']['share_of_step'],4), round(d['tree_roofline']['expand']['ms']/max(1,d['tree_roofline']['expand']['dispatches'])*1e3,1))")"
  done
done
