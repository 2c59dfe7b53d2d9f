"""Busy time of the trunk kernel from a rocprofv3 kernel trace (scripts/gpu_prof_bench.sh).

With L lanes (bench.py --lanes, engine.LanedEngine) the L k_tower_dyn dispatches of one simulation
step run concurrently, so bench.py reports roofline.avg_launch_us = union busy time of all
k_tower_dyn dispatches / (dispatches / L).  This recomputes the same figure from rocprof's own
start/end timestamps, beside rocprof's per-dispatch average (= bench.py's avg_dispatch_us).
`last` (optional): keep only the last N dispatches (the bench's timed region: bench.py reports its
roofline.dispatches), so warm-up plies - with leaf dedup, early plies have far fewer rows - do not
enter the averages.
"""
import csv
import json
import sys


def main(trace_csv, lanes, out_json, last=0, kernel="k_tower_dyn"):
    lanes, last = int(lanes), int(last)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(trace_csv))
                if kernel in r["Kernel_Name"])
    if last > 0:
        iv = iv[-last:]
    busy, cs, ce = 0, None, None
    for a, b in iv:
        if ce is None or a > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    if ce is not None:
        busy += ce - cs
    n = len(iv)
    res = dict(kernel=kernel, dispatches=n, lanes=lanes,
               avg_dispatch_us=sum(b - a for a, b in iv) / max(1, n) / 1e3,
               union_busy_ms=busy / 1e6,
               avg_launch_us=busy / max(1, n // lanes) / 1e3,
               note="avg_launch_us = union of the dispatch intervals / (dispatches / lanes), as bench.py "
                    "roofline.avg_launch_us; avg_dispatch_us = rocprof's per-dispatch mean")
    json.dump(res, open(out_json, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:5])
