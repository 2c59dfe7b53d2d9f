# BASELINE config 3 (Connect4, 800 sims, 16,384 games per GPU, ResNet-256x20) in steady state: warm-up of
# one game generation (WARM plies, ~42), then STEPS timed plies, then TWIN plies of the same games with
# leaf dedup off (bench.py --twin-no-dedup: every leaf its own row, as the reference).  The node store is
# recycled (k_compact) at BPT blocks per tree, default 8,000 (2,000 exhausts it in steady state; the high-water is ~6,000).  EXTRA
# passes more bench flags.  Progress lines go to the .err file (one per warm-up ply).
set -u
mkdir -p gpurun_out/cfg3
export TMPDIR=/tmp
TAG=${TAG:-dedup}
timeout -k 10 ${T:-1100} python3 -u bench.py --games 16384 --sims 800 --filter-factor 64 --warmup ${WARM:-42} \
  --steps ${STEPS:-6} --blocks-per-tree ${BPT:-8000} --twin-no-dedup ${TWIN:-4} --no-cpu-baseline --progress ${EXTRA:-} \
  > gpurun_out/cfg3/config3_steady_$TAG.json 2> gpurun_out/cfg3/config3_steady_$TAG.err
rc=$?; echo "config3 $TAG rc=$rc"; tail -3 gpurun_out/cfg3/config3_steady_$TAG.err
[ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/cfg3/config3_steady_$TAG.json') if l.startswith('{')][0]); print(round(d['value'],1), d['roofline']['frac'], d['nn']['rows_per_leaf'], d['tree']['blocks_in_use_max'], d['tree']['compactions'], d.get('no_dedup_twin'))"
