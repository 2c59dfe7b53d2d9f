#!/bin/bash
# Round-5 G6 extension (build container only: imports /root/reference).  21 parts of 1,000 reference
# threaded searches (ResNet-128x20, 200 sims, thread_count 4, one game thread), LANES processes side by
# side at one thread each, niced; then merged into tests/golden/threaded_stats.json.
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
OUTD=${OUTD:-/tmp/g6r5}
LANES=${LANES:-6}
mkdir -p "$OUTD"
jobs=()
for pi in 0 1 2; do for c in 0 1 2; do jobs+=("$pi:$c"); done; done
for pi in 3 4 5; do for c in 0 1 2 3; do jobs+=("$pi:$c"); done; done
run_lane() {
  local lane=$1
  local i=0
  for j in "${jobs[@]}"; do
    if (( i % LANES == lane )); then
      pi=${j%%:*}; c=${j##*:}
      f="$OUTD/part_${pi}_${c}.json"
      if [ ! -s "$f" ]; then
        OMP_NUM_THREADS=1 nice -n 19 python "$HERE/make_threaded_stats.py" resnet_single 1000 "$pi" "$f.tmp" \
          > "$OUTD/log_${pi}_${c}.txt" 2>&1 && mv "$f.tmp" "$f"
      fi
    fi
    i=$((i + 1))
  done
}
for l in $(seq 0 $((LANES - 1))); do run_lane "$l" & done
wait
ls "$OUTD"/part_*.json | wc -l
