"""Effective clock and MFMA-pipe utilisation of k_tower launches from one rocprofv3 PMC pass
(scripts/gpu_tower_util.sh).  GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md
'DVFS give-back'); SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-busy cycles summed over all SIMDs."""
import collections
import csv
import json
import sys

SIMDS = 256 * 4


def main(path, out, last="0"):
    """`last` > 0: the last N dispatches only (a bench command's timed region), aggregated over their
    summed cycles (clock_ghz / mfma_busy_frac of all of them together) as well as per dispatch."""
    last = int(last)
    disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        d = disp[int(r["Dispatch_Id"])]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    ids = sorted(disp)
    if last > 0:
        ids = ids[-last:]
    sel = [disp[i] for i in ids]
    rows = []
    for d in sel:
        cyc = d["GRBM_GUI_ACTIVE"] / 8
        row = dict(ns=d["ns"], clock_ghz=cyc / d["ns"],
                   mfma_busy_frac=d["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * SIMDS))
        if "SQ_INSTS_MFMA" in d:
            row["mfma_insts"] = d["SQ_INSTS_MFMA"]
        if "SQ_WAVE_CYCLES" in d:  # disjoint split of wave cycles (MI355X_MICROARCH.md PMC slots)
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY"):
                if k in d:
                    row[k.lower()[3:] + "_frac"] = d[k] / d["SQ_WAVE_CYCLES"]
        if "SQ_LDS_IDX_ACTIVE" in d:
            row["lds_bank_conflict_frac"] = d.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(d["SQ_LDS_IDX_ACTIVE"], 1.0)
            row["lds_active_frac"] = d["SQ_LDS_IDX_ACTIVE"] / (cyc * 256)
        rows.append(row)
    if last <= 0:
        rows = rows[2:] or rows  # skip warm-up dispatches
        sel = sel[2:] or sel
    n = len(rows)
    res = {k: sum(r[k] for r in rows) / n for k in rows[0]}
    cyc = sum(d["GRBM_GUI_ACTIVE"] / 8 for d in sel)
    res["clock_ghz_weighted"] = cyc / sum(d["ns"] for d in sel)
    res["mfma_busy_frac_weighted"] = sum(d["SQ_VALU_MFMA_BUSY_CYCLES"] for d in sel) / (cyc * SIMDS)
    res["dispatches"] = n
    res["note"] = ("per-dispatch means, and cycle-weighted over the dispatches (_weighted); "
                   "clock = GRBM_GUI_ACTIVE / 8 / duration; mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / "
                   "(cycles x 1024 SIMDs); `last` > 0: a bench command's timed dispatches only")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(*sys.argv[1:4])
