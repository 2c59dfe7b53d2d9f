"""Idle / tower-free time of a rocprofv3 kernel trace of bench.py (profiles/r02_ss/): over the last
`plies` plies (k_games_begin_ply marks, one per lane), the time no kernel runs and the time no
k_tower_dyn runs, with the kernels that run in the tower-free windows.

    python scripts/trace_idle.py run_kernel_trace.csv [plies] [lanes]
"""
import collections
import csv
import json
import sys


def union(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def main(path, plies=7, lanes=2):
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("<")[0][:48])
                for r in csv.DictReader(open(path)))
    begins = [e[0] for e in ev if "k_games_begin_ply" in e[2]]
    start = begins[-int(plies) * int(lanes)]
    sub = [e for e in ev if e[0] >= start]
    end = max(e[1] for e in sub)
    busy = union([(s, e) for s, e, _ in sub])
    tower = union([(s, e) for s, e, n in sub if "k_tower_dyn" in n])
    span = end - start
    free, t = [], start
    for s, e in tower:
        if s > t:
            free.append((t, s))
        t = max(t, e)
    if end > t:
        free.append((t, end))
    att = collections.Counter()
    for a, b in free:
        for s, e, n in sub:
            o = min(b, e) - max(a, s)
            if o > 0:
                att[n] += o
    # windows by ply phase: one holding a k_select_vl (the first fill of a ply's searches), one holding
    # the ply-end kernels (move choice, finish / refill), or a simulation step's window (expand / leaf rows)
    cls = collections.Counter()
    ncls = collections.Counter()
    durs = []
    for a, b in free:
        names = {n for s, e, n in sub if min(b, e) - max(a, s) > 0}
        k = ("ply_start" if any("k_select_vl" in n for n in names) else
             "ply_end" if any("k_games" in n for n in names) else "sim_step")
        cls[k] += b - a
        ncls[k] += 1
        durs.append((b - a) / 1e3)
    durs.sort()
    q = lambda f: durs[min(len(durs) - 1, int(f * len(durs)))] if durs else 0.0
    res = dict(span_ms=span / 1e6, idle_frac=1 - sum(e - s for s, e in busy) / span,
               tower_free_frac=sum(b - a for a, b in free) / span, tower_free_windows=len(free),
               window_us_quantiles={"p10": q(0.1), "p50": q(0.5), "p90": q(0.9), "max": q(1.0)},
               by_phase_frac={k: v / span for k, v in cls.items()}, by_phase_windows=dict(ncls),
               overlapping_kernels_ms={k: v / 1e6 for k, v in att.most_common(8)})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
