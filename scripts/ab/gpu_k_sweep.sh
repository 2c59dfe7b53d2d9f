set -o pipefail
cd $GRAFT_REPO_ROOT
for k in 2 8; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --search-threads $k > gpurun_out/sweep_k$k.json 2> gpurun_out/sweep_k$k.err || exit $?
done
timeout -k 10 300 python -u bench.py --no-cpu-baseline --search-threads 4 --lanes 1 > gpurun_out/sweep_k4_l1.json 2> gpurun_out/sweep_k4_l1.err
