# Round 5: speculative child-block prefetch in sim_vl (ab_libs/libspmcts_pf.so = the tree) vs the same tree
# without it (ab_libs/libspmcts_nopf.so), one box: Philox games identical (scripts/rng_equal.py), isolated
# steady-state tree kernels alternated, the driver-form bench alternated.
set -u
O=gpurun_out/r05i
mkdir -p $O
export TMPDIR=/tmp
PF=$PWD/ab_libs/libspmcts_pf.so
NOPF=$PWD/ab_libs/libspmcts_nopf.so
SPMCTS_LIB=$PF timeout -k 10 300 python3 scripts/rng_equal.py $O/rng_pf.npz > $O/rng.log 2>&1 || { tail -5 $O/rng.log; exit 1; }
SPMCTS_LIB=$NOPF timeout -k 10 300 python3 scripts/rng_equal.py $O/rng_nopf.npz >> $O/rng.log 2>&1 || { tail -5 $O/rng.log; exit 1; }
python3 scripts/rng_equal.py --compare $O/rng_pf.npz $O/rng_nopf.npz | tee -a $O/summary.txt
for rep in 1 2; do
  for v in pf nopf; do
    if [ $v = pf ]; then LIB=$PF; else LIB=$NOPF; fi
    SPMCTS_LIB=$LIB timeout -k 10 300 python3 scripts/bench_tree.py --warmup 24 --plies 8 > $O/iso_${v}_$rep.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    echo "iso steady $v: $(python3 -c "import json; d=json.loads(open('$O/iso_${v}_$rep.json').read().strip().splitlines()[-1]); print({k: (round(v, 1) if isinstance(v, float) else v) for k, v in d.items() if k in ('select_avg_us', 'expand_avg_us', 'ply_ms')})")" | tee -a $O/summary.txt
  done
done
for rep in 1 2; do
  for v in pf nopf; do
    if [ $v = pf ]; then LIB=$PF; else LIB=$NOPF; fi
    SPMCTS_LIB=$LIB timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline --twin-no-dedup 0 > $O/b_${v}_$rep.json 2>$O/err.txt || { tail -5 $O/err.txt; exit 1; }
    echo "bench $v: $(python3 -c "import json; d=json.loads([l for l in open('$O/b_${v}_$rep.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['tree_roofline']['avg_launch_us'],1))")" | tee -a $O/summary.txt
  done
done
exit 0
