"""How many of a simulation step's network rows (already deduplicated within the step) hold a position that
an EARLIER step evaluated: the hit rate a cross-step evaluation cache (a transposition table over leaf
planes) would have.  One SelfPlayEngine (no lanes), the bench's network and search settings (ResNet-128x20,
torch.manual_seed(0), fp16, 200 sims, K = 4, leaf dedup on); each step's rows are read back (host sync:
a diagnostic, not a bench), hashed from their planes and looked up in
  * `ply`: the rows of the earlier steps of the same ply,
  * `prev_ply`: the rows of the same ply and the previous one,
  * `all`: every row since the start.
Prints one JSON line per ply and a summary over the plies after --warmup.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch

from self_play_reinforcement_learning_amd.engine import SelfPlayEngine
from self_play_reinforcement_learning_amd.modules import ResidualTower

ap = argparse.ArgumentParser()
ap.add_argument("--games", type=int, default=4096)
ap.add_argument("--plies", type=int, default=25)
ap.add_argument("--warmup", type=int, default=5)
ap.add_argument("--sims", type=int, default=200)
ap.add_argument("--threads", type=int, default=4)
args = ap.parse_args()
dev = torch.device("cuda:0")
torch.manual_seed(0)
net = ResidualTower(7, 6, 7, num_blocks=20, filter_factor=32).to(dev).eval()
eng = SelfPlayEngine("connect4", net, n_games=args.games, iterations=args.sims, seed=1234, device=dev,
                     search_threads=args.threads, dtype=torch.float16)
a = eng.arena
W1 = (2 ** torch.arange(63, dtype=torch.int64, device=dev))


def keys(n):
    x = a._leaves[:n].reshape(n, -1)  # the rows' planes as the network reads them
    bits = (x != 0).to(torch.int64)
    assert bits.shape[1] <= 189, bits.shape
    pad = torch.zeros((n, 189 - bits.shape[1]), dtype=torch.int64, device=dev)
    bits = torch.cat([bits, pad], 1).reshape(n, 3, 63)
    k = (bits * W1).sum(2)  # three exact 63-bit words
    return k[:, 0] * 1000003 ^ k[:, 1] * 998244353 ^ k[:, 2]  # 64-bit mix (collisions ~ n^2 / 2^64)


def member(sorted_seen, k):
    if sorted_seen.numel() == 0:
        return torch.zeros_like(k, dtype=torch.bool)
    i = torch.searchsorted(sorted_seen, k).clamp(max=sorted_seen.numel() - 1)
    return sorted_seen[i] == k


def merge(sorted_seen, k):
    return torch.unique(torch.cat([sorted_seen, k]))


seen_all = torch.empty(0, dtype=torch.int64, device=dev)
seen_prev = torch.empty(0, dtype=torch.int64, device=dev)
tot = dict(rows=0, ply=0, prev_ply=0, all=0)
eng.start()
for p in range(args.plies):
    eng._ply_begin()
    seen_ply = torch.empty(0, dtype=torch.int64, device=dev)
    st = dict(rows=0, ply=0, prev_ply=0, all=0)

    for i in range(eng.select_steps + 1):
        if i < eng.select_steps:
            eng._ply_sim_net(i)
        else:
            a.games_end_ply_async()
            eng._eval_dev(cap=2 * eng.n_games)
        torch.cuda.synchronize()
        n = int(a.count_dev[0].item())
        if n:
            k = keys(n)
            hp = member(seen_ply, k)
            hpp = hp | member(seen_prev, k)
            ha = member(seen_all, k)
            st["rows"] += n
            st["ply"] += int(hp.sum())
            st["prev_ply"] += int(hpp.sum())
            st["all"] += int(ha.sum())
            seen_ply = merge(seen_ply, k)
            seen_all = merge(seen_all, k)
        eng._expand_dev(sim=i < eng.select_steps)
    eng._ply_finish()
    seen_prev = seen_ply
    line = dict(ply=p, rows=st["rows"], **{f"hit_{w}": round(st[w] / max(1, st["rows"]), 4) for w in ("ply", "prev_ply", "all")},
                cache_entries=int(seen_all.numel()), games_done=eng.games_done)
    print(json.dumps(line), flush=True)
    if p >= args.warmup:
        for w in tot:
            tot[w] += st[w]
print(json.dumps({"summary": True, "plies": args.plies - args.warmup, "rows": tot["rows"],
                  **{f"hit_{w}": round(tot[w] / max(1, tot["rows"]), 4) for w in ("ply", "prev_ply", "all")}}))
