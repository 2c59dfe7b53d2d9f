# Same-box A/B of lane scheduling variants on the default bench workload (steady state: 24 warm-up plies).
set -u
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
A="--warmup 24 --steps ${STEPS:-40} --no-cpu-baseline"
for v in base prio lanes3 base2 prio2; do
  case $v in
    base|base2) E=""; X="";;
    prio|prio2) E="SPMCTS_LANE_PRIORITY=1"; X="";;
    lanes3) E=""; X="--lanes 3";;
  esac
  env $E timeout -k 10 300 python3 bench.py $A $X > gpurun_out/ab/$v.json 2> gpurun_out/ab/$v.err
  rc=$?; echo "$v rc=$rc $(python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab/$v.json') if l.startswith('{')][0]); print(round(d['value']), round(d['roofline']['frac'],4), round(d['nn']['share_of_step'],4))")"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab/$v.err; exit $rc; fi
done
