# Same-box A/B of two builds of the library on the full bench (alternating runs): LIBS="a.so b.so".
set -u
mkdir -p gpurun_out/bab
export TMPDIR=/tmp
: > gpurun_out/bab/ab.txt
for rep in 1 2; do
  for lib in ${LIBS}; do
    SPMCTS_LIB=$PWD/self_play_reinforcement_learning_amd/$lib timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bab/one.json 2> gpurun_out/bab/err.txt
    rc=$?; if [ $rc -ne 0 ]; then echo "lib $lib rc=$rc"; tail -3 gpurun_out/bab/err.txt; exit $rc; fi
    python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/bab/one.json') if l.startswith('{')][0]); print(sys.argv[1], round(d['value'],1), round(d['roofline']['frac'],4), round(d['tree_roofline']['avg_launch_us'],2))" $lib | tee -a gpurun_out/bab/ab.txt
  done
done
