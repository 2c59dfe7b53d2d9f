# Round-2 verification of the current tree: full -m gpu suite, smoke, default bench, then the
# bench's rocprof evidence (kernel trace + FETCH/WRITE_SIZE passes) via gpu_prof_bench.sh.
set -u
mkdir -p gpurun_out/ver
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/ver/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ver/gpu_tests.log; if [ $rc -ne 0 ]; then grep -E "FAIL|Error" gpurun_out/ver/gpu_tests.log | head -20; exit $rc; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/ver/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/ver/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > gpurun_out/ver/bench.json 2> gpurun_out/ver/bench.err
rc=$?; cut -c1-400 gpurun_out/ver/bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/ver/bench.err; exit $rc; }
[ "${PROF:-1}" = 1 ] && bash scripts/gpu_prof_bench.sh
