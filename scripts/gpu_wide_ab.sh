# One-buffer C = 256 trunk (tower_wide.h) vs the 3-board two-buffer tiles (default; SPMCTS_TOWER_C256=6 selects the one-buffer tiles), one box:
# bit-equality of both paths' outputs (host batch + device-count ragged batch; C = 128 against the
# previous build), the tower GPU tests, then alternating trunk-only timings at ResNet-256x20.
set -u
mkdir -p gpurun_out/wide
export TMPDIR=/tmp
O=gpurun_out/wide
L=$PWD/self_play_reinforcement_learning_amd
SPMCTS_TOWER_C256=3 timeout -k 10 300 python3 scripts/tower_code_equal.py dump $O/c3.npz 64 &&
SPMCTS_TOWER_C256=6 timeout -k 10 300 python3 scripts/tower_code_equal.py dump $O/wide.npz 64 || exit 1
python3 scripts/tower_code_equal.py cmp $O/c3.npz $O/wide.npz || [ "${NOEQ:-0}" = 1 ] || exit 1
SPMCTS_LIB=$L/libspmcts_prev.so timeout -k 10 300 python3 scripts/tower_code_equal.py dump $O/p128.npz 32 &&
timeout -k 10 300 python3 scripts/tower_code_equal.py dump $O/n128.npz 32 || exit 1
python3 scripts/tower_code_equal.py cmp $O/p128.npz $O/n128.npz || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_tower.py -x -q -m gpu --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error|assert" $O/tests.log | head; exit $rc; fi
for BATCH in ${WBATCH:-1536 6144}; do
  for rep in 1 2; do
    for c in 3 6; do
      SPMCTS_TOWER_C256=$c timeout -k 10 120 python3 scripts/bench_tower.py --trunk-only --ff 64 --batch $BATCH --iters 10 > $O/one.json 2>$O/err.txt || { tail -3 $O/err.txt; exit 1; }
      echo "trunk C=256 $BATCH tiles $c: $(python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), 'us', round(d['tflops'],1), 'TF/s')")"
    done
  done
done
