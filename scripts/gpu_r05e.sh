# Kernel trace of the graphed trainer step with the HIP block convolutions (per-kernel stats only).
set -u
O=gpurun_out/r05e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d /tmp/r05e_prof -o run -- python3 scripts/bench_train.py --trainer-only-graph > $O/prof.json 2> $O/prof.err || { tail -5 $O/prof.err; exit 1; }
find /tmp/r05e_prof -name "*kernel_stats.csv" -exec cp {} $O/trainer_step_kernel_stats.csv \;
rm -rf /tmp/r05e_prof
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r05e/trainer_step_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f'{100*float(r["TotalDurationNs"])/tot:5.1f} % {int(r["Calls"]):6d} {float(r["AverageNs"])/1e3:8.1f} us {r["Name"][:110]}')
PY
exit 0
