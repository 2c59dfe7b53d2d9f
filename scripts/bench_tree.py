"""Tree kernels in isolation: the threaded (K sims in flight) select / expand kernels of one arena of
`games` Connect4 games, `sims` sims/move, with the device table net as the leaf evaluator (so no
tower dispatch shares the chip with them), timed with HIP events around each launch on the arena's
stream.  Prints one JSON line: per-kernel average duration and the algorithmic bytes / achieved GB/s
of bench.py's byte models (select_bytes + expand_bytes).

    python scripts/bench_tree.py [--games 4096] [--sims 200] [--threads 4] [--plies 4]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=4096)
    ap.add_argument("--sims", type=int, default=200)
    ap.add_argument("--threads", type=int, default=4)
    ap.add_argument("--plies", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--blocks-per-tree", type=int, default=0,
                    help="node store per tree (0 = the worst case, no recycling; below it k_compact recycles)")
    ap.add_argument("--prof", action="store_true",
                    help="with SPMCTS_LIB=.../libspmcts_prof.so (make prof): shader-clock cycles per sim phase")
    args = ap.parse_args()
    import torch

    import bench
    from self_play_reinforcement_learning_amd.arena import Arena, table_net_eval
    from self_play_reinforcement_learning_amd.engine import EventTimer

    G, K = args.games, args.threads
    a = Arena("connect4", n_trees=2 * G, n_games=G, iterations=args.sims, rng="philox", seed=5, leaf_format="f32",
              search_threads=K, blocks_per_tree=args.blocks_per_tree)
    a.games_set_limit(-1)
    a.games_start(list(range(G)))
    steps = -(-args.sims // K)
    ts, te = EventTimer(), EventTimer()

    def ev(n):
        return table_net_eval("connect4", a.leaves(n), "f32", "nchw", salt=7)

    def ply(timed):
        a.games_begin_ply()
        for i in range(steps):
            if i == 0 or K == 1:
                n = a.select(ts if timed else None)  # the timer brackets the select kernel alone
            else:
                a.leaf_rows_async()
                n = int(a.count_dev.cpu()[0])
            if n:
                p, v = ev(n)
                if timed:
                    te.start()
                a.expand(p, v)
                if timed:
                    te.stop()
        n = a.games_end_ply()
        if n:
            p, v = ev(n)
            a.expand(p, v)
        a.games_finish_ply(refill=True)

    for _ in range(args.warmup):
        ply(False)
    prof = None
    if args.prof:
        import ctypes

        prof = ctypes.CDLL(os.environ["SPMCTS_LIB"]).spmcts_ab_tree_prof
        prof.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
        buf = (ctypes.c_ulonglong * 16)()
        torch.cuda.synchronize()
        assert prof(buf, 1) == 0
    c0 = a.counters()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.plies):
        ply(True)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    a.check()
    c1 = a.counters()
    sims = c1["sims"] - c0["sims"]
    levels = c1["depth_sum"] - c0["depth_sum"]
    nn = c1["nn_leaves"] - c0["nn_leaves"]
    sel_b = bench.select_bytes(sims, levels, threads=K)
    exp_b = bench.expand_bytes(nn, levels * nn / max(1, sims), threads=K)
    t_s, t_e = ts.total_ms(), te.total_ms()
    out = dict(games=G, sims=args.sims, threads=K, plies=args.plies, select_dispatches=ts.count(),
               expand_dispatches=te.count(), select_avg_us=t_s / max(1, ts.count()) * 1e3,
               expand_avg_us=t_e / max(1, te.count()) * 1e3, tree_bytes=sel_b + exp_b,
               achieved_gbs=(sel_b + exp_b) / ((t_s + t_e) / 1e3) / 1e9, mean_levels=levels / max(1, sims),
               nn_leaves=nn, sims_done=sims, blocks_per_tree=a.blocks_per_tree, ply_ms=wall / args.plies * 1e3,
               compactions=c1["compactions"] - c0["compactions"], blocks_in_use_max=c1["blocks_in_use_max"])
    out["frac_of_8tbs"] = out["achieved_gbs"] / 8000.0
    if prof is not None:
        assert prof(buf, 1) == 0
        names = ("load", "score", "argmax", "leaf", "descend", "rng")
        for base, kern in ((0, "select"), (8, "expand")):
            tot = sum(buf[base + i] for i in range(6))
            out[f"prof_{kern}"] = dict({n: round(buf[base + i] / max(1, tot), 4) for i, n in enumerate(names)},
                                       phase_cycles=tot, max_launch_cycles=buf[base + 6], max_sims=buf[base + 7])
        out["prof_cycles_per_sim"] = (sum(buf[i] for i in range(6)) + sum(buf[8 + i] for i in range(6))) / max(1, sims)
        out["prof_cycles_per_level"] = (sum(buf[i] for i in range(6)) + sum(buf[8 + i] for i in range(6))) / max(1, levels)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
