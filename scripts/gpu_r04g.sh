# Round 4 pass g: kernel breakdown of the graphed trainer step (gpu_trainer_prof.sh), the driver-form
# bench with the fp16 and the bf16 trunk alternated on one box (the dtype gap like for like), then the
# staggered-lanes A/B with the reordered issue (gpu_stagger_ab.sh, SKIP_TESTS=1).
set -u
export TMPDIR=/tmp
bash scripts/gpu_trainer_prof.sh || exit $?
O=gpurun_out/dtype_ab
mkdir -p $O
for rep in 1 2; do
  for dt in fp16 bf16; do
    timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline --twin-no-dedup 0 --dtype $dt > $O/b_${dt}_$rep.json 2> $O/err.txt || { tail -5 $O/err.txt; exit 1; }
    echo "bench $dt: $(python3 -c "import json; d=json.loads([l for l in open('$O/b_${dt}_$rep.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_us'],1), round(d['nn']['share_of_step'],4))")" | tee -a $O/summary.txt
  done
done
SKIP_TESTS=1 bash scripts/gpu_stagger_ab.sh
