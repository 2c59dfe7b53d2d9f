#!/bin/bash
# Round-6 G6 evaluate-mode set (build container only: imports /root/reference).  The reference's threaded
# search with MCTreeSearch.evaluate(True) (BASELINE config 5's arena search): ResNet-128x20 seed 0, 200 sims,
# thread_count 4, one game thread, 1,200 searches at each of 5 G6 positions, one process per position at
# one thread each, niced; then merged into tests/golden/threaded_stats.json as `resnet_eval`.
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
OUTD=${OUTD:-/tmp/g6r6}
N=${N:-1200}
mkdir -p "$OUTD"
for pi in 0 1 3 4 5; do
  f="$OUTD/eval_${pi}.json"
  if [ ! -s "$f" ]; then
    ( OMP_NUM_THREADS=1 nice -n 19 python "$HERE/make_threaded_stats.py" resnet_eval "$N" "$pi" "$f.tmp" \
        > "$OUTD/log_eval_${pi}.txt" 2>&1 && mv "$f.tmp" "$f" ) &
  fi
done
wait
python "$HERE/make_threaded_stats.py" merge resnet_eval "$OUTD"/eval_*.json
