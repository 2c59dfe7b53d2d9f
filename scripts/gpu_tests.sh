# GPU test pass: the listed test files (default: all -m gpu), one process, own time limit.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 ${T:-900} python -m pytest ${FILES:-tests} -m gpu -x -q ${PYARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -30 gpurun_out/gpu_tests.log
exit $rc
