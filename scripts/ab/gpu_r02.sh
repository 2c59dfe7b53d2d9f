# Round-2 GPU pass: the -m gpu suite (one process, per-test timeout), smoke, default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu ${PYARGS:-} > gpurun_out/r02_gpu_tests.log 2>&1 && \
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02_smoke.log 2>&1 && \
timeout -k 10 400 python -u bench.py ${BENCHARGS:-} > gpurun_out/r02_bench.json 2> gpurun_out/r02_bench.err
rc=$?
tail -5 gpurun_out/r02_gpu_tests.log
cut -c1-400 gpurun_out/r02_bench.json 2>/dev/null
exit $rc
