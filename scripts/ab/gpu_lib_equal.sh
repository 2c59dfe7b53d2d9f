# Bit-equality of two builds of the library on the host-path trunk + heads (LIBS="a.so b.so"),
# then the tower GPU tests on the default build.
set -u
mkdir -p gpurun_out/eq
export TMPDIR=/tmp
set -- ${LIBS}
SPMCTS_LIB=$PWD/self_play_reinforcement_learning_amd/$1 timeout -k 10 180 python scripts/tower_code_equal.py dump gpurun_out/eq/a.npz &&
SPMCTS_LIB=$PWD/self_play_reinforcement_learning_amd/$2 timeout -k 10 180 python scripts/tower_code_equal.py dump gpurun_out/eq/b.npz &&
python scripts/tower_code_equal.py cmp gpurun_out/eq/a.npz gpurun_out/eq/b.npz &&
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_tower.py > gpurun_out/tower_tests.log 2>&1; rc=$?; tail -2 gpurun_out/tower_tests.log; exit $rc
