# A timing alternative (SPMCTS_TOWER_CG=$CODE) against the default trunk on one box: bit-equality of
# the outputs (scripts/tower_code_equal.py), then alternating trunk timings at 4,096 boards.
set -u
mkdir -p gpurun_out/eq
export TMPDIR=/tmp
timeout -k 10 180 python scripts/tower_code_equal.py dump gpurun_out/eq/a.npz &&
SPMCTS_TOWER_CG=$CODE timeout -k 10 120 python scripts/tower_code_equal.py dump gpurun_out/eq/b.npz &&
python scripts/tower_code_equal.py cmp gpurun_out/eq/a.npz gpurun_out/eq/b.npz &&
PAIRS="\"d\":2 \"x\":$CODE \"d\":2 \"x\":$CODE \"d\":2 \"x\":$CODE" BATCH=4096 bash scripts/gpu_tower_codes.sh
