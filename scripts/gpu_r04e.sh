# Round 4 pass e: search-shift diagnostic (scripts/diag/shift_excess.py), the driver-form bench and the
# trainer throughput (gpu_r04.sh stages bench + train), then the weight-major MFMA order probe.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
timeout -k 10 400 python3 -u scripts/diag/shift_excess.py > gpurun_out/diag/shift_excess.json 2> gpurun_out/diag/shift_excess.err
rc=$?; cat gpurun_out/diag/shift_excess.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/diag/shift_excess.err; exit $rc; }
STAGES="bench train" bash scripts/gpu_r04.sh || exit $?
bash scripts/gpu_codes_clock_ab.sh
