# Round 4 pass d: C = 256 buffer-resource scratch fix (gpu_c256_rsrc_fix.sh) and the trainer determinism
# diagnostic with deterministic convolution algorithms requested.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/diag
timeout -k 10 300 python3 scripts/diag/trainer_determinism.py --deterministic > gpurun_out/diag/trainer_det2.json 2> gpurun_out/diag/trainer_det2.err
rc=$?; cat gpurun_out/diag/trainer_det2.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/diag/trainer_det2.err; exit $rc; }
bash scripts/gpu_c256_rsrc_fix.sh
