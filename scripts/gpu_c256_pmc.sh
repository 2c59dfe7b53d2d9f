# C = 256 trunk (config 3's ResNet-256x20): PMC comparison of the shipped 3-board two-buffer tiles and
# the 6-board one-buffer edge tiles (SPMCTS_TOWER_C256=6, tower_wide.h), trunk-only micro-benchmark at
# 6,144 boards: clock, MFMA busy and instruction counts (pass 1), wave-cycle split and LDS (pass 2).
# One rocprofv3 pass per run, each under its own time limit.
set -u
O=gpurun_out/c256pmc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_tower.py -x -q -m gpu -k "wide_c256 or coresident" --timeout 250 \
  --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/tests.log | head; exit $rc; }
for rep in 1 2; do
  for c in 3 6; do
    SPMCTS_TOWER_C256=$c timeout -k 10 120 python3 scripts/bench_tower.py --trunk-only --ff 64 --batch 6144 --iters 10 > $O/one.json 2>$O/err.txt || { tail -3 $O/err.txt; exit 1; }
    echo "trunk C=256 6144 tiles $c: $(python3 -c "import json; d=json.loads(open('$O/one.json').read().strip().splitlines()[-1]); print(round(d['trunk_ms']*1e3,1), 'us', round(d['tflops'],1), 'TF/s')")" | tee -a $O/timing.txt
  done
done
P1="GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
P2="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT"
for tiles in 3 6; do
  i=0
  for set in "$P1" "$P2"; do
    i=$((i+1))
    SPMCTS_TOWER_C256=$tiles timeout -s KILL 150 rocprofv3 --pmc $set --kernel-include-regex "k_tower" -f csv \
      -d $O/t${tiles}_p$i -o run -- python3 scripts/bench_tower.py --trunk-only --iters 6 --batch 6144 --ff 64 \
      > $O/t${tiles}_p$i.json 2> $O/t${tiles}_p$i.err
    rc=$?; echo "tiles $tiles pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/t${tiles}_p$i.err; exit $rc; }
    python3 scripts/tower_util.py $O/t${tiles}_p$i/run_counter_collection.csv $O/util_t${tiles}_p$i.json
  done
done
python3 - <<'EOF'
import csv, collections, json
O = "gpurun_out/c256pmc"
for tiles in (3, 6):
    tot = collections.Counter()
    n = collections.Counter()
    for i in (1, 2):
        disp = collections.defaultdict(dict)
        for r in csv.DictReader(open(f"{O}/t{tiles}_p{i}/run_counter_collection.csv")):
            d = disp[int(r["Dispatch_Id"])]
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        ids = sorted(disp)[2:]  # skip warm-up dispatches
        for j in ids:
            for k, v in disp[j].items():
                tot[f"p{i}:{k}"] += v
            n[i] += 1
    avg = {k: v / n[int(k[1])] for k, v in tot.items()}
    print(tiles, json.dumps({k: round(v, 1) for k, v in sorted(avg.items())}))
EOF
