# Round-3 closing pass, one box: the session-start library vs the final one on the driver-form bench
# (alternated, REPS rounds; bit-equality of the trunk outputs first), then config 3 after one game
# generation with its no-dedup twin (scripts/gpu_config3_steady.sh).  The first failure ends the call.
set -u
LIBS="libspmcts_start.so libspmcts.so" REPS=${REPS:-2} bash scripts/gpu_bench_libs_ab.sh || exit $?
T=${T3:-800} TAG=dedup bash scripts/gpu_config3_steady.sh
