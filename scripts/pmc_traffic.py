"""Per-launch L2<->fabric traffic of the trunk kernel from rocprofv3 PMC passes (scripts/gpu_prof_bench.sh).

FETCH_SIZE / WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of 16-B-per-lane
streaming reads (MI355X_MICROARCH.md, HBM/rocprofv3 section), so reads are doubled.  Writes the
JSON that bench.py reports as roofline.traffic.
"""
import csv
import json
import sys


def mean_counter(path, name, kernel="k_tower_dyn", last=0):
    """Mean per dispatch (counter rows summed per dispatch); `last` > 0 keeps the last N dispatches
    (the bench's timed region, after its warm-up plies)."""
    per = {}
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == name:
            d = int(r["Dispatch_Id"])
            per[d] = per.get(d, 0.0) + float(r["Counter_Value"])
    vals = [per[d] for d in sorted(per)]
    if last > 0:
        vals = vals[-last:]
    return sum(vals) / len(vals), len(vals)


def main(fetch_csv, write_csv, out_json, lanes="1", last="0", kernel="k_tower_dyn"):
    """`kernel`: a substring of the kernel name (k_tower for the host-count trunk of scripts/bench_tower.py)."""
    lanes, last = int(lanes), int(last)
    fetch, n = mean_counter(fetch_csv, "FETCH_SIZE", kernel=kernel, last=last)
    write, _ = mean_counter(write_csv, "WRITE_SIZE", kernel=kernel, last=last)
    per_dispatch = 2 * fetch * 1024 + write * 1024
    res = dict(kernel=kernel, dispatches=n, lanes=lanes, fetch_kib=fetch, write_kib=write,
               read_bytes=2 * fetch * 1024, write_bytes=write * 1024,
               bytes_per_dispatch=per_dispatch,
               bytes_per_launch=per_dispatch * lanes,
               note="per dispatch: FETCH_SIZE x2 (gfx950 16-B read correction) + WRITE_SIZE, KiB -> bytes; "
                    "L2<->fabric traffic (Infinity Cache hits included); a launch = `lanes` concurrent "
                    "dispatches (bench.py roofline)")
    json.dump(res, open(out_json, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:7])
