#!/bin/bash
# Product device code before/after a source refactor (round 6: the Cfg::ABL ablations moved out of the product
# k-loops into tower_abl.h / tower_m16_abl.h): the gfx950 assembly of one translation unit with the product
# flags (no -DSPMCTS_AB), comments and debug directives stripped, compared with a saved copy.  Only the
# per-compilation __hip_cuid_* symbol may differ.  Runs on the build host (no GPU).
#   scripts/product_isa_equal.sh save tower.hip /tmp/base.s     (before)
#   scripts/product_isa_equal.sh cmp  tower.hip /tmp/base.s     (after)
set -e
mode=$1; src=$2; ref=$3
cd "$(dirname "$0")/../self_play_reinforcement_learning_amd/csrc"
out=$(mktemp)
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -std=c++17 -fPIC -ffp-contract=off -fno-gpu-rdc -I../../include \
  --offload-device-only -S "$src" -o "$out.raw" 2>/dev/null
grep -v '^\s*;' "$out.raw" | sed 's/\s*;.*$//' | grep -v '^\s*\.\(file\|loc\|ident\)' | grep -v 'amdhsa.version\|\.amdgcn_target\|^\s*$' \
  | grep -v '__hip_cuid_' > "$out"
rm -f "$out.raw"
if [ "$mode" = save ]; then mv "$out" "$ref"; echo "saved $(wc -l < "$ref") lines, $(grep -c s_endpgm "$ref") kernels"; exit 0; fi
if cmp -s "$out" "$ref"; then echo "identical: $(wc -l < "$ref") lines, $(grep -c s_endpgm "$ref") kernels"; rm -f "$out"; exit 0; fi
diff "$ref" "$out" | head -20; rm -f "$out"; exit 1
