"""Per-kernel reduction of one rocprofv3 PMC pass (counter_collection.csv): for every kernel name, the
dispatch count, mean duration, effective clock (GRBM_GUI_ACTIVE / 8 / duration, MI355X_MICROARCH.md 'DVFS
give-back'), MFMA-busy share (SQ_VALU_MFMA_BUSY_CYCLES over 1,024 SIMDs) and the disjoint split of the waves'
cycles (SQ_WAIT_ANY parked / SQ_WAIT_INST_ANY issue-stalled / SQ_ACTIVE_INST_ANY issuing), cycle-weighted over
the dispatches.  rocprofv3 serialises the dispatches it counts, so kernels that overlap in an unprofiled run
(the bench's two lanes) are measured one at a time here.

    python scripts/pmc_per_kernel.py counter_collection.csv out.json [name-regex]
"""
import collections
import csv
import json
import re
import sys

SIMDS = 256 * 4


def main(path, out, pat="."):
    rx = re.compile(pat)
    disp = collections.defaultdict(dict)
    names = {}
    for r in csv.DictReader(open(path)):
        i = int(r["Dispatch_Id"])
        d = disp[i]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        names[i] = r["Kernel_Name"]
    by = collections.defaultdict(list)
    for i, d in disp.items():
        short = re.sub(r"\(.*", "", names[i])
        if rx.search(short):
            by[short[:90]].append(d)
    res = {}
    for k, ds in sorted(by.items(), key=lambda kv: -sum(d["ns"] for d in kv[1])):
        ns = sum(d["ns"] for d in ds)
        cyc = sum(d.get("GRBM_GUI_ACTIVE", 0.0) / 8 for d in ds)
        row = dict(dispatches=len(ds), mean_us=ns / len(ds) / 1e3, total_ms=ns / 1e6,
                   clock_ghz=cyc / ns if ns else None)
        if cyc and any("SQ_VALU_MFMA_BUSY_CYCLES" in d for d in ds):
            row["mfma_busy_frac"] = sum(d.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for d in ds) / (cyc * SIMDS)
        wc = sum(d.get("SQ_WAVE_CYCLES", 0.0) for d in ds)
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                row[c.lower()[3:] + "_frac"] = sum(d.get(c, 0.0) for d in ds) / wc
        # every other counter: its mean per dispatch (and, for SQ_ cycle / wait / active counters, its share
        # of the waves' cycles)
        for c in sorted({c for d in ds for c in d if c not in ("ns",)}):
            if c in ("GRBM_GUI_ACTIVE", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                     "SQ_ACTIVE_INST_ANY"):
                continue
            tot = sum(d.get(c, 0.0) for d in ds)
            row[c.lower() + "_per_dispatch"] = tot / len(ds)
            if wc and c.startswith("SQ_") and c != "SQ_WAVE_CYCLES" and ("CYCLES" in c or "WAIT" in c or "ACTIVE" in c):
                row[c.lower()[3:] + "_frac"] = tot / wc
        res[k] = row
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res.items():
        print(k[:60], {a: (round(b, 4) if isinstance(b, float) else b) for a, b in v.items()})


if __name__ == "__main__":
    main(*sys.argv[1:4])
