# BASELINE configs beside the headline: config 3 (800 sims, 16,384 games, ResNet-256x20) on the recycled
# node store, and config 5 (arena evaluation) in steady state (warm-up past the longest game).
set -u
mkdir -p gpurun_out/cfg
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --mode arena --games 8192 --warmup ${AW:-45} --steps ${AS:-40} --no-cpu-baseline > gpurun_out/cfg/config5_arena_steady.json 2> gpurun_out/cfg/c5.err
rc=$?; echo "arena rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/cfg/c5.err; exit $rc; fi
grep '^{' gpurun_out/cfg/config5_arena_steady.json | cut -c1-300
timeout -k 10 400 python3 -u bench.py --games 16384 --sims 800 --filter-factor 64 --warmup 2 --steps 4 --blocks-per-tree 1800 --no-cpu-baseline > gpurun_out/cfg/config3_recycled.json 2> gpurun_out/cfg/c3.err
rc=$?; echo "config3 rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/cfg/c3.err; exit $rc; fi
grep '^{' gpurun_out/cfg/config3_recycled.json | cut -c1-300
