# Round 4 pass f: the profile bundle of the final tree (gpu_prof_r04.sh: bench trace + trunk traffic, tree
# traffic, in-bench clock / MFMA busy of both trunk dtypes), then the multi-rank rehearsal (self-launched and
# torchrun 2-rank gloo on the one GPU, the RCCL one-rank group) with the per-rank report.
set -u
export TMPDIR=/tmp
bash scripts/gpu_prof_r04.sh || exit $?
bash scripts/gpu_multirank_final.sh
