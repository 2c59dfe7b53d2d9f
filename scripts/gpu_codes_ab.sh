# Trunk timing alternatives (SPMCTS_TOWER_CG codes in $CODES, the first is the reference) on one box:
# bit-equality of each code's outputs with the first's (scripts/tower_code_equal.py; NOEQ=1 only
# prints the comparison), then alternating trunk-only timings at one and four workgroup rounds.
set -u
mkdir -p gpurun_out/codes
export TMPDIR=/tmp
O=gpurun_out/codes
set -- $CODES
REF=$1
SPMCTS_TOWER_CG=$REF timeout -k 10 180 python3 scripts/tower_code_equal.py dump $O/ref.npz || exit 1
for c in "$@"; do
  [ "$c" = "$REF" ] && continue
  SPMCTS_TOWER_CG=$c timeout -k 10 180 python3 scripts/tower_code_equal.py dump $O/c$c.npz || exit 1
  echo "code $c vs $REF: $(python3 scripts/tower_code_equal.py cmp $O/ref.npz $O/c$c.npz)"
  python3 scripts/tower_code_equal.py cmp $O/ref.npz $O/c$c.npz > /dev/null || [ "${NOEQ:-0}" = 1 ] || exit 1
done
for BATCH in ${BATCHES:-1536 6144}; do
  for rep in 1 2 3; do
    for c in "$@"; do
      SPMCTS_TOWER_CG=$c timeout -k 10 120 python3 scripts/bench_tower.py --trunk-only --batch $BATCH --iters 30 > $O/one.json 2>$O/err.txt || { tail -3 $O/err.txt; exit 1; }
      echo "trunk $BATCH code $c: $(python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), 'us', round(d['tflops'],1), 'TF/s')")"
    done
  done
done
