# Round 5: the tree-kernel alternates of the A/B library play the product's games bit for bit.
set -u
O=gpurun_out/r05w
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_tree_alternates.py -m gpu -x -v --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -5 $O/tests.log; exit $rc
