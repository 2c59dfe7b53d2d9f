# Round 6: (1) the vendor GEMM's rate on the same box as the fused trunk, each with its own clock
# (scripts/gemm_ceiling.py); (2) the hit rate a cross-step evaluation cache would have on the bench's workload
# (scripts/diag/leaf_cache_hits.py: rows of a step whose planes an earlier step evaluated).
set -u
O=gpurun_out/r06j
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python3 scripts/gemm_ceiling.py --reps 3 > $O/gemm_ceiling.json 2> $O/gemm_ceiling.err
rc=$?; echo "gemm_ceiling rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/gemm_ceiling.err; exit $rc; }
python3 -c "
import json; d=json.loads(open('$O/gemm_ceiling.json').read().strip().splitlines()[-1])
for k, v in d['runs'].items(): print(k, [(r['tflops'], r['frac'], r['clock_ghz'], r['frac_at_clock']) for r in v])" | tee $O/summary.txt
timeout -k 10 600 python3 -u scripts/diag/leaf_cache_hits.py --plies 30 --warmup 5 > $O/leaf_cache_hits.jsonl 2> $O/leaf_cache_hits.err
rc=$?; echo "leaf_cache_hits rc=$rc"; tail -4 $O/leaf_cache_hits.jsonl | tee -a $O/summary.txt; [ $rc -eq 0 ] || { tail -20 $O/leaf_cache_hits.err; exit $rc; }
exit 0
