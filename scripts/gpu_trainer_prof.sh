# Kernel breakdown of the graphed trainer step (batch 64, ResNet-128x20, fp16 autocast, train mode):
# rocprofv3 kernel trace + stats of scripts/bench_train.py's trainer-only timing, top kernels by time.
set -u
O=gpurun_out/trainprof
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- \
  python3 scripts/bench_train.py --trainer-only-graph > $O/out.json 2> $O/err.txt
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/err.txt; exit $rc; }
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/trainprof/trace/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("kernels", len(rows), "total ms", round(tot / 1e6, 2))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(round(float(r["TotalDurationNs"]) / tot * 100, 1), "%", r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us", r["Name"][:110])
PY
