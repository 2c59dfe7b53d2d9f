# C = 256 residual scratch through a buffer resource with soffset-free stores (the shipped form, tower_wide.h
# ScrBuf) against the round-3 pointer form: (1) the C = 256 tower tests (3-board vs 6-board tiles bit for bit,
# fp32 tolerance), (2) host-path outputs of the product library vs the A/B library's pointer form (CG 2566),
# (3) trunk-only timings at 6,144 boards, alternated, (4) config 3 (ResNet-256x20, 800 sims, 16,384 games,
# plies 3-6) on the product library vs the previous product library (lib_c256ptr.so), alternated.
set -u
O=gpurun_out/c256fix
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/self_play_reinforcement_learning_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_tower.py -m gpu -x -q --timeout 400 --timeout-method thread > $O/tower_tests.log 2>&1
rc=$?; tail -2 $O/tower_tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/tower_tests.log | head -60; exit $rc; }
SPMCTS_LIB=$L/libspmcts.so timeout -k 10 240 python3 scripts/tower_code_equal.py dump $O/rsrc.npz 64 || exit 1
SPMCTS_LIB=$L/libspmcts_ab.so SPMCTS_TOWER_CG=2566 timeout -k 10 240 python3 scripts/tower_code_equal.py dump $O/ptr.npz 64 || exit 1
echo "rsrc vs pointer: $(python3 scripts/tower_code_equal.py cmp $O/rsrc.npz $O/ptr.npz)" | tee -a $O/summary.txt
for rep in 1 2; do
  for v in rsrc ptr; do
    if [ $v = rsrc ]; then env="SPMCTS_LIB=$L/libspmcts.so"; else env="SPMCTS_LIB=$L/libspmcts_ab.so SPMCTS_TOWER_CG=2566"; fi
    env $env timeout -k 10 120 python3 scripts/bench_tower.py --trunk-only --ff 64 --batch 6144 --iters 10 > $O/one.json 2>$O/err.txt || { tail -3 $O/err.txt; exit 1; }
    echo "trunk C256 6144 $v $(python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), round(d['tflops'],1))")" | tee -a $O/summary.txt
  done
done
if [ "${SKIP_C3:-0}" != 1 ]; then
for rep in 1 2; do
  for lib in libspmcts.so lib_c256ptr.so; do
    SPMCTS_LIB=$L/$lib timeout -k 10 400 python3 -u bench.py --games 16384 --sims 800 --filter-factor 64 --warmup 3 \
      --steps 4 --blocks-per-tree 2000 --no-cpu-baseline --twin-no-dedup 0 --no-secondary > $O/c3_$lib.json 2> $O/c3_$lib.err || { tail -5 $O/c3_$lib.err; exit 1; }
    echo "config3 $lib: $(python3 -c "import json; d=json.loads([l for l in open('$O/c3_$lib.json') if l.startswith('{')][0]); print(round(d['value'],1), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4))")" | tee -a $O/summary.txt
  done
done
fi
exit 0
