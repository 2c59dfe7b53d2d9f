# k_expand_vl held to 96 registers (SPMCTS_EXPAND_CO=1: fits beside a trunk wave, with spills) vs the
# default: threaded parity under the variant, then same-box bench A/B, short and steady state.
set -u
mkdir -p gpurun_out/eco
export TMPDIR=/tmp
SPMCTS_EXPAND_CO=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k threaded --timeout 120 --timeout-method thread > gpurun_out/eco/parity.log 2>&1
rc=$?; tail -1 gpurun_out/eco/parity.log; if [ $rc -ne 0 ]; then exit $rc; fi
for W in "5 20" "24 40"; do
  set -- $W
  for C in 0 1 0 1; do
    SPMCTS_EXPAND_CO=$C timeout -k 10 300 python3 bench.py --warmup $1 --steps $2 --no-cpu-baseline > gpurun_out/eco/b.json 2>gpurun_out/eco/err.txt || { tail -3 gpurun_out/eco/err.txt; exit 1; }
    echo "bench w$1 expand_co $C: $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/eco/b.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4), round(d['tree_roofline']['expand']['ms']/max(1,d['tree_roofline']['expand']['dispatches'])*1e3,1))")"
  done
done
