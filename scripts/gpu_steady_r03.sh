# Round-3 steady-state evidence, one box: (1) a rocprofv3 kernel trace of the bench after one game
# generation of warm-up (42 plies, 7 timed plies) and the tower-free share of its last 7 plies
# (scripts/trace_idle.py); (2) train_model throughput (scripts/bench_train.py: trainer stream on / off,
# fp16 autocast / fp32); (3) config 3's C = 256 linear heads, co-resident vs LDS-staged, alternated.
# Own time limit per step; the first failure ends the call.
set -u
O=gpurun_out/steady
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- \
  python3 bench.py --warmup 42 --steps 7 --no-cpu-baseline > $O/bench_traced.json 2> $O/trace.err
rc=$?; echo "steady trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/trace.err; exit $rc; }
python3 scripts/trace_idle.py $O/trace/run_kernel_trace.csv 7 2 > $O/trace_idle.json && cat $O/trace_idle.json
rm -f $O/trace/run_kernel_trace.csv.gz
if [ "${SKIP_TRAIN:-0}" != 1 ]; then
timeout -k 10 600 python3 -u scripts/bench_train.py > $O/train.json 2> $O/train.err
rc=$?; echo "train rc=$rc"; cut -c1-2500 $O/train.json; [ $rc -eq 0 ] || { tail -20 $O/train.err; exit $rc; }
fi
[ "${SKIP_C3:-0}" = 1 ] && exit 0
for rep in 1 2; do
  for h in co lds; do
    SPMCTS_HEADS_C256=$h timeout -k 10 400 python3 -u bench.py --games 16384 --sims 800 --filter-factor 64 --warmup 3 \
      --steps 4 --blocks-per-tree 2000 --no-cpu-baseline > $O/c3_$h.json 2> $O/c3_$h.err || { tail -5 $O/c3_$h.err; exit 1; }
    echo "config3 heads $h: $(python3 -c "import json; d=json.loads([l for l in open('$O/c3_$h.json') if l.startswith('{')][0]); print(round(d['value'],1), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4))")" | tee -a $O/c3_heads_ab.txt
  done
done
exit 0
