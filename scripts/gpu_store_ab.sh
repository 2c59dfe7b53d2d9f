# Node-store change vs the previous build (libspmcts_prev.so): identical games in Philox mode
# (scripts/rng_equal.py), the parity / engine GPU tests on the new build, isolated tree kernels and a
# bench A/B (short run), alternated.  Own time limit per step; the first failure ends the call.
set -u
mkdir -p gpurun_out/st
export TMPDIR=/tmp
O=gpurun_out/st
L=$PWD/self_play_reinforcement_learning_amd
SPMCTS_LIB=$L/libspmcts_prev.so timeout -k 10 200 python3 scripts/rng_equal.py $O/prev.npz > $O/eq.log 2>&1 || { tail -5 $O/eq.log; exit 1; }
SPMCTS_LIB=$L/libspmcts.so timeout -k 10 200 python3 scripts/rng_equal.py $O/new.npz >> $O/eq.log 2>&1 || { tail -5 $O/eq.log; exit 1; }
python3 scripts/rng_equal.py --compare $O/prev.npz $O/new.npz || exit 1
timeout -k 10 ${T:-700} python -u -m pytest ${FILES:-tests/test_gpu_parity.py tests/test_gpu_engine.py} -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head; exit $rc; fi
for rep in 1 2; do
  for lib in libspmcts_prev.so libspmcts.so; do
    SPMCTS_LIB=$L/$lib timeout -k 10 120 python3 scripts/bench_tree.py > $O/iso.json 2>$O/err.txt || { tail -3 $O/err.txt; exit 1; }
    echo "iso $lib: $(python3 -c "import json; d=json.loads(open('$O/iso.json').read().strip().splitlines()[-1]); print(round(d['select_avg_us'],1), round(d['expand_avg_us'],1))")"
  done
done
for rep in 1 2; do
  for lib in libspmcts_prev.so libspmcts.so; do
    SPMCTS_LIB=$L/$lib timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline > $O/b.json 2>$O/err.txt || { tail -3 $O/err.txt; exit 1; }
    echo "bench w5 $lib: $(python3 -c "import json; d=json.loads([l for l in open('$O/b.json') if l.startswith('{')][0]); print(round(d['value']), round(d['nn']['share_of_step'],4), round(d['tree_roofline']['expand']['ms']/max(1,d['tree_roofline']['expand']['dispatches'])*1e3,1))")"
  done
done
