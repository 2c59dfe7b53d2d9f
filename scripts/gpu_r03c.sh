# Round-3 pass 3 (session 3): the whole -m gpu suite on the current tree, smoke, the driver-form bench,
# then config 3 (ResNet-256x20, 800 sims, 16,384 games) with the C = 256 linear heads co-resident
# (two-pass k_heads_co) vs LDS-staged (SPMCTS_HEADS_C256=lds), alternated.  Own time limit per step.
set -u
O=gpurun_out/r03c
mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 ${T:-900} python -u -m pytest ${FILES:-tests} -m gpu -x -v --timeout 400 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed" $O/gpu_tests.log | tail -2; [ $rc -eq 0 ] || { grep -B5 -A30 "FAILED\|Error" $O/gpu_tests.log | head -80; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.loads([l for l in open('$O/bench.json') if l.startswith('{')][0]); print('bench', round(d['value']), round(d['roofline']['frac'],4), d['cpu_baseline']['value'])"
[ "${1:-}" = SKIPC3 ] && exit 0
for rep in 1 2; do
  for h in co lds; do
    SPMCTS_HEADS_C256=$h timeout -k 10 400 python3 -u bench.py --games 16384 --sims 800 --filter-factor 64 --warmup 3 \
      --steps 4 --blocks-per-tree 2000 --no-cpu-baseline > $O/c3_$h.json 2> $O/c3_$h.err || { tail -5 $O/c3_$h.err; exit 1; }
    echo "config3 heads $h: $(python3 -c "import json; d=json.loads([l for l in open('$O/c3_$h.json') if l.startswith('{')][0]); print(round(d['value'],1), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4))")" | tee -a $O/c3_heads_ab.txt
  done
done
exit 0
