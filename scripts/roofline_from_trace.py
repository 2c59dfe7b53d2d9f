"""Recompute a bench line's trunk roofline from the rocprofv3 kernel trace of the SAME run.

    python scripts/roofline_from_trace.py <bench_line.json> <run_kernel_trace.csv[.gz]> <out.json>

The traced command prints its own bench.py JSON line (HIP-event timing: roofline.avg_launch_us, .frac,
.flops_per_launch over roofline.dispatches k_tower_dyn dispatches of the timed region).  Here the same
dispatches are taken from the trace (the last `dispatches` k_tower_dyn records: the bench's timed region
comes after its warm-up plies, and the profiled form runs no dispatches after it, --twin-no-dedup 0),
their union busy time is divided into launches of `lanes` concurrent dispatches as bench.py does, and
the frac is recomputed from the line's own FLOPs per launch:

    frac_trace = flops_per_launch / (union_busy / launches) / peak

DESIGN.md §5 states the two side by side; they must agree within 2 %.
"""
import csv
import gzip
import json
import sys


def union_us(iv):
    busy, cs, ce = 0, None, None
    for a, b in sorted(iv):
        if ce is None or a > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    if ce is not None:
        busy += ce - cs
    return busy / 1e3


def main(line_json, trace_csv, out_json, kernel="k_tower_dyn"):
    line = json.loads([l for l in open(line_json) if l.startswith("{")][0])
    rf = line["roofline"]
    n, lanes = int(rf["dispatches"]), int(rf["lanes"])
    f = gzip.open(trace_csv, "rt") if trace_csv.endswith(".gz") else open(trace_csv)
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(f) if kernel in r["Kernel_Name"])
    if len(iv) < n:
        raise SystemExit(f"trace holds {len(iv)} {kernel} dispatches, the line {n}")
    iv = iv[-n:]
    launches = n // lanes
    launch_us = union_us(iv) / launches
    tflops = rf["flops_per_launch"] / (launch_us * 1e-6) / 1e12
    frac = tflops / rf["peak"]
    res = dict(kernel=kernel, dispatches=n, lanes=lanes, launches=launches,
               avg_dispatch_us_trace=sum(b - a for a, b in iv) / n / 1e3,
               avg_dispatch_us_events=rf["avg_dispatch_us"],
               avg_launch_us_trace=launch_us, avg_launch_us_events=rf["avg_launch_us"],
               flops_per_launch=rf["flops_per_launch"], peak_tflops=rf["peak"],
               tflops_trace=tflops, frac_trace=frac, frac_events=rf["frac"],
               frac_ratio_trace_over_events=frac / rf["frac"],
               executed_frac_trace=frac * rf["executed"]["flops_per_leaf"] / rf["flops_per_leaf"]
               if rf.get("executed") else None,
               clock=rf.get("clock"), value=line["value"], ms_per_step=line["ms_per_step"],
               note="one run: the HIP-event roofline of the traced command's own bench line vs the same "
                    "dispatches' rocprofv3 kernel-trace timestamps (union busy per launch of `lanes` dispatches)")
    json.dump(res, open(out_json, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:5])
