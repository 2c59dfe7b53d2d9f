"""Per-dispatch L2<->fabric traffic of the tree kernels (k_select_vl + k_expand_vl) from rocprofv3 PMC
passes over the bench command (scripts/gpu_prof_tree.sh).  FETCH_SIZE doubled (gfx950 16-B read
correction, MI355X_MICROARCH.md), KiB -> bytes.  bench.py reports bytes_per_dispatch as
tree_roofline.traffic (its algorithmic bytes are per dispatch of either kernel as well)."""
import csv
import json
import sys

KERNELS = ("k_select_vl", "k_expand_vl")


def per_kernel(path, name, last=0):
    """Counter per dispatch of each tree kernel; `last` > 0 keeps the last N tree dispatches (both
    kernels together, dispatch order: the bench's timed region)."""
    per = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != name:
            continue
        for k in KERNELS:
            if k in r["Kernel_Name"]:
                d = int(r["Dispatch_Id"])
                kk, v = per.get(d, (k, 0.0))
                per[d] = (k, v + float(r["Counter_Value"]))
    ids = sorted(per)
    if last > 0:
        ids = ids[-last:]
    out = {k: [] for k in KERNELS}
    for d in ids:
        out[per[d][0]].append(per[d][1])
    return out


def main(fetch_csv, write_csv, out_json, last="0"):
    f = per_kernel(fetch_csv, "FETCH_SIZE", int(last))
    w = per_kernel(write_csv, "WRITE_SIZE", int(last))
    res = dict(kernels={})
    tot_bytes, tot_n = 0.0, 0
    for k in KERNELS:
        n = len(f[k])
        if not n:
            continue
        rb, wb = 2 * 1024 * sum(f[k]), 1024 * sum(w[k])
        res["kernels"][k] = dict(dispatches=n, read_bytes_per_dispatch=rb / n,
                                 write_bytes_per_dispatch=wb / max(1, len(w[k])))
        tot_bytes += rb + wb * n / max(1, len(w[k]))
        tot_n += n
    res["bytes_per_dispatch"] = tot_bytes / max(1, tot_n)
    res["dispatches"] = tot_n
    res["note"] = ("mean over every k_select_vl and k_expand_vl dispatch of the traced bench run: FETCH_SIZE x2 + "
                   "WRITE_SIZE, KiB -> bytes (L2<->fabric, Infinity Cache hits included)")
    json.dump(res, open(out_json, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:5])
