# With leaf dedup and the co-resident heads: one arena (bigger dedup pool, no lane overlap) vs two lanes.
set -u
mkdir -p gpurun_out/ld
export TMPDIR=/tmp
for W in "5 20" "24 40"; do
  set -- $W
  for L in 2 1 2 1; do
    timeout -k 10 300 python3 bench.py --warmup $1 --steps $2 --lanes $L --no-cpu-baseline > gpurun_out/ld/b.json 2>gpurun_out/ld/err.txt || { tail -3 gpurun_out/ld/err.txt; exit 1; }
    echo "bench w$1 lanes $L: $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ld/b.json') if l.startswith('{')][0]); n=d['nn']; print(round(d['value']), round(d['roofline']['frac'],4), round(n['share_of_step'],4), round(n['rows_per_leaf'],4))")"
  done
done
