# The graphed trainer step (batch 64, ResNet-128x20) under MIOpen solver restrictions: MIOpen picks its
# dot2 Winograd kernels (miopenSp3AsmConv ... fp16_dot2 ... f2x3: VALU dot products, no MFMA; 46 % of the
# step, scripts/gpu_trainer_prof.sh) for the 3x3 convs; with them disabled it falls back to other solvers.
set -u
O=gpurun_out/trainmi
mkdir -p $O
export TMPDIR=/tmp
run() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python3 -u scripts/bench_train.py --trainer-only-graph > $O/$tag.json 2> $O/$tag.err || { tail -5 $O/$tag.err; return 1; }
  echo "$tag: $(python3 -c "import json; d=json.loads(open('$O/$tag.json').read().strip().splitlines()[-1]); print([round(r['ms_per_sgd_step'],2) for r in d['trainer_only']])")" | tee -a $O/summary.txt
}
run default A=1 || exit 1
run no_rxs_f2x3 MIOPEN_DEBUG_AMD_WINOGRAD_RXS_F2X3=0 || exit 1
run no_rxs MIOPEN_DEBUG_AMD_WINOGRAD_RXS_F2X3=0 MIOPEN_DEBUG_AMD_WINOGRAD_RXS_F3X2=0 || exit 1
run no_winograd MIOPEN_DEBUG_AMD_WINOGRAD_RXS_F2X3=0 MIOPEN_DEBUG_AMD_WINOGRAD_RXS_F3X2=0 MIOPEN_DEBUG_AMD_WINOGRAD_RXS=0 MIOPEN_DEBUG_AMD_WINOGRAD_3X3=0 MIOPEN_DEBUG_AMD_FUSED_WINOGRAD=0 || exit 1
run no_winograd_no_naive MIOPEN_DEBUG_AMD_WINOGRAD_RXS_F2X3=0 MIOPEN_DEBUG_AMD_WINOGRAD_RXS_F3X2=0 MIOPEN_DEBUG_AMD_WINOGRAD_RXS=0 MIOPEN_DEBUG_AMD_WINOGRAD_3X3=0 MIOPEN_DEBUG_AMD_FUSED_WINOGRAD=0 MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD=0 MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_BWD=0 MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_WRW=0 || exit 1
exit 0
