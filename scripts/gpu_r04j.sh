# Final-tree pass: the GPU tests, smoke and the driver-form bench (scripts/gpu_r04.sh), then the bench's
# trunk dtype A/B on the same box (fp16, the default, vs bf16; alternated, twice).
set -u
STAGES="tests bench" bash scripts/gpu_r04.sh || exit $?
O=gpurun_out/r04j
mkdir -p $O
for rep in 1 2; do
  for dt in fp16 bf16; do
    timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline --twin-no-dedup 0 --dtype $dt > $O/b_${dt}_$rep.json 2>$O/err.txt || { tail -5 $O/err.txt; exit 1; }
    echo "bench $dt: $(python3 -c "import json; d=json.loads([l for l in open('$O/b_${dt}_$rep.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['roofline']['avg_launch_us'],1))")"
  done
done
exit 0
