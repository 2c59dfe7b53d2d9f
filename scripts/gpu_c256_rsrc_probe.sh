# Which half of the buffer-resource residual-scratch form gives the different C = 256 outputs:
# trunk outputs of the 2- and 20-block ResNet-256 (scripts/tower_code_equal.py, host path) of the product
# library's pointer form against the A/B library's SPMCTS_TOWER_CG probes 2561 (rsrc loads + stores, nt),
# 2563 (rsrc loads, pointer stores), 2564 (pointer loads, rsrc stores), 2565 (rsrc loads + stores, sc0 sc1).
set -u
O=gpurun_out/rsrc_probe
mkdir -p $O
export TMPDIR=/tmp
L=$PWD/self_play_reinforcement_learning_amd
SPMCTS_LIB=$L/libspmcts.so timeout -k 10 240 python3 scripts/tower_code_equal.py dump $O/ref.npz 64 || exit 1
for code in ${CODES:-2561 2563 2564 2565}; do
  SPMCTS_LIB=$L/libspmcts_ab.so SPMCTS_TOWER_CG=$code timeout -k 10 240 python3 scripts/tower_code_equal.py dump $O/x$code.npz 64 || exit 1
  echo "code $code: $(python3 scripts/tower_code_equal.py cmp $O/ref.npz $O/x$code.npz)" | tee -a $O/summary.txt
done
