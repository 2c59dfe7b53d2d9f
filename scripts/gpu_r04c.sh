# trainer determinism diagnostic, then pass b (rsrc probes + steady trace)
set -u
mkdir -p gpurun_out/diag
timeout -k 10 300 python3 scripts/diag/trainer_determinism.py > gpurun_out/diag/trainer_det.json 2> gpurun_out/diag/trainer_det.err
rc=$?; cat gpurun_out/diag/trainer_det.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/diag/trainer_det.err; exit $rc; }
bash scripts/gpu_r04b.sh
