"""G6: statistics of the reference's THREADED search, produced by running the reference itself.

Run in the build container only (needs /root/reference):

    python tests/golden/make_threaded_stats.py [table|resnet|resnet_seq|all]

The reference searches with `thread_count` concurrent search_node calls per tree and
virtual loss whenever its network is an InferenceProxy (games/algos/mcts.py:154,
:328-331, :340-367) — the default of SelfPlayScheduler.train_model
(self_play_parallel.py:95-171).  Those threads interleave nondeterministically, so no
single threaded search can be a bit-exact fixture; what the reference does pin is the
DISTRIBUTION of search outcomes.  This script reproduces the reference's own serving
structure, using the reference's classes unchanged:

  * one QueueContainer(threading=threads_per_worker * thread_count) → one InferenceProxy
    (self_play_parallel.py:102-108);
  * the reference's InferenceWorker (inference_worker.py:89-119) started as its own
    process, polling the queues and batching whatever requests are present;
  * `threads_per_worker` game threads (selfplayworker.py:101-138), each running
    MCTreeSearch(network=proxy, thread_count=4) searches on fixed positions reached by
    play_action (mcts.py:188-209), then `_play(1)` (mcts.py:272-299).

Per search it records the Move's tree_probs (the root visit distribution at temperature
1), the chosen action and the root q.  The GPU test (tests/test_gpu_statistical.py)
compares the Philox arena's K=4 search against these samples with a stated tolerance.

Sets (200 sims, thread_count 4 unless stated):
  table_serving / table_single    the deterministic table net (oracle/table_net.py) served
              through the InferenceWorker, with 8 game threads sharing the worker's queue pool
              (the reference's default threads_per_worker) or with one game thread;
  resnet_serving / resnet_single  ResidualTower(7, 6, 7, num_blocks=20, filter_factor=32),
              random init torch.manual_seed(0) (the bench's ResNet-128x20), same two regimes;
  resnet_seq  the same net called directly (no proxy: the reference's sequential mode) —
              the K=1 counterpart at the headline net and budget.

Each position also records how many expansions re-expanded an already expanded node: the
threaded search checks `is_leaf` before taking the node's lock (mcts.py:357-359), so two
threads can expand the same leaf and the second replaces the first one's children.  With
one game thread this is rare; with 8 game threads contending for the GIL it is frequent,
and it measurably flattens the root visit distribution.

Round 6: resnet_eval is the arena's search (BASELINE config 5): the same threaded pipeline with
`MCTreeSearch.evaluate(True)` on both the tree and its _play — root noise still on (mcts.py:323-327), the
move drawn from n^20 (temp/20, mcts.py:273-276; selfplayworker.py:71-81 sets evaluate on both arena
policies).  Each sample also records the root visit counts.  Made in parts by tests/golden/run_g6_eval.sh
and merged with `merge resnet_eval <parts...>`.

Only inputs and the outputs the reference produced are written (no reference source).

Round 3: resnet_single holds 1,000 searches per position (was 160), made with one process per
position side by side (OMP_NUM_THREADS=2 each) and merged:

    for p in 0 1 2; do OMP_NUM_THREADS=2 python tests/golden/make_threaded_stats.py \
        resnet_single 1000 $p /tmp/g6_rs_$p.json & done; wait
    python tests/golden/make_threaded_stats.py merge resnet_single /tmp/g6_rs_{0,1,2}.json

Round 5: resnet_single holds 4,000 searches at each of 6 positions (3,000 more at positions 0-2, 4,000
at the new positions 3-5), made in 1,000-search parts by tests/golden/run_g6_parts.sh (one thread per
part process, six parts side by side) and merged with `merge_append resnet_single <parts...>`.
"""
import concurrent.futures
import json
import os
import sys
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
OUT = os.path.join(HERE, "threaded_stats.json")

sys.path.insert(0, os.path.join(HERE, "refshims"))
sys.path.insert(0, REF)
sys.path.insert(0, REPO)

import torch  # noqa: E402

from oracle.table_net import cells_of, table_eval  # noqa: E402

POSITIONS = [[], [3, 3, 2], [2, 4, 3, 3, 1],
             [3], [3, 2, 4, 4], [2, 3, 3, 4, 4, 2]]  # round 5: positions 3-5 added
SIMS = 200
THREADS = 4          # thread_count (mcts.py:131 default)
GAME_THREADS = 8     # threads_per_worker (self_play_parallel.py:95 default)
TABLE_SALT = 4242


class TableNetModule(torch.nn.Module):
    """The table net with the batched `forward(LongTensor[B, W, H]) -> (probs[B, A], v[B, 1])`
    surface InferenceWorker.calculate expects (inference_worker.py:114-119).  Rows arrive
    already multiplied by the mover (inference_proxy.py:21-24)."""

    def __init__(self, n_actions, salt):
        super().__init__()
        self.n_actions, self.salt = n_actions, salt

    def forward(self, batch):
        ps, vs = [], []
        for row in batch.numpy():
            p, v = table_eval(cells_of(row), self.n_actions, self.salt)
            ps.append(p)
            vs.append([v])
        return torch.tensor(np.array(ps, np.float32)), torch.tensor(np.array(vs, np.float32))


def _resnet():
    from games.general.modules import ResidualTower

    torch.manual_seed(0)
    net = ResidualTower(width=7, height=6, action_size=7, num_blocks=20, filter_factor=32)
    net.eval()
    sd = net.state_dict()
    return net, {k: float(v.double().sum()) for k, v in sd.items()}


def _search_once(MCTreeSearch, Connect4Env, network, opening, thread_count, evaluate=False):
    tree = MCTreeSearch(network=network, env=Connect4Env, iterations=SIMS, thread_count=thread_count)
    for a in opening:
        tree.play_action(a, None)
    tree.train(False)
    tree.evaluate(evaluate)
    action = tree()
    mv = tree.temp_memory[-1]
    out = dict(tree_probs=mv.tree_probs.numpy().astype(float).tolist(), action=int(action), q=float(mv.q),
               root_n=int(tree.root_node.n))
    if evaluate:  # tree_probs are n^20 there (mcts.py:273-276): keep the visit counts as well
        out["visits"] = [int(c.n) for c in tree.root_node.children]
    return out


class _ReexpansionCounter:
    """Observation only: counts MCNode.create_children calls on nodes that already have children.
    In threaded mode search_node checks `child.is_leaf` before `child.lock.acquire` (mcts.py:357-359),
    so two threads can both pass the check; the second then re-expands the node, replacing the
    first thread's children (create_children rebinds `children`, mcts.py:103-107).  How often this
    happens depends on how the host schedules the threads (GIL contention), so it is recorded."""

    def __init__(self):
        from games.algos import mcts as ref_mcts

        self.cls, self.orig = ref_mcts.MCNode, ref_mcts.MCNode.create_children
        self.calls = self.re = 0
        counter = self

        def wrapped(node, probs, valid):
            counter.calls += 1
            if node.children:
                counter.re += 1
            return counter.orig(node, probs, valid)

        self.cls.create_children = wrapped

    def close(self):
        self.cls.create_children = self.orig
        return dict(expansions=self.calls, re_expansions=self.re)


def run_threaded(net_module, samples, label, game_threads, positions=POSITIONS, evaluate=False):
    """The reference's serving structure: InferenceWorker process + proxy + game threads."""
    from games.algos.inference_proxy import InferenceProxy
    from games.algos.inference_worker import InferenceWorker
    from games.algos.mcts import MCTreeSearch
    from games.connect4.connect4env import Connect4Env
    from rl_utils.queues import QueueContainer

    queue = QueueContainer(threading=game_threads * THREADS)
    proxy = InferenceProxy(queue.policy_queues)
    worker = InferenceWorker([queue], net_module, save_dir="/tmp/g6_saves", start_time="g6")
    worker.daemon = True
    worker.start()
    out = []
    lock = threading.Lock()
    t0 = time.time()
    try:
        for opening in positions:
            counter = _ReexpansionCounter()
            res = []

            def job(_):
                r = _search_once(MCTreeSearch, Connect4Env, proxy, opening, THREADS, evaluate)
                with lock:
                    res.append(r)
                    if len(res) % 20 == 0:
                        print(f"  {label} {opening}: {len(res)}/{samples} ({time.time() - t0:.0f} s)", flush=True)

            with concurrent.futures.ThreadPoolExecutor(game_threads) as ex:
                list(ex.map(job, range(samples)))
            out.append(dict(opening=opening, samples=res, **counter.close()))
    finally:
        worker.terminate()
        worker.join()
    return out


def _seq_job(args):
    opening, seeds = args
    torch.set_num_threads(1)
    from games.algos.mcts import MCTreeSearch
    from games.connect4.connect4env import Connect4Env

    net, _ = _resnet()
    res = []
    with torch.no_grad():
        for s in seeds:
            np.random.seed(s)
            res.append(_search_once(MCTreeSearch, Connect4Env, net, opening, 4))  # direct net: sequential
    return res


def run_sequential(samples, procs=8):
    import multiprocessing as mp

    out = []
    for pi, opening in enumerate(POSITIONS):
        seeds = [70_000 + 1000 * pi + i for i in range(samples)]
        chunks = [(opening, seeds[i::procs]) for i in range(procs)]
        with mp.get_context("spawn").Pool(procs) as pool:
            res = [r for part in pool.map(_seq_job, chunks) for r in part]
        out.append(dict(opening=opening, samples=res))
        print(f"  resnet_seq {opening}: {len(res)} searches", flush=True)
    return out


def _rounded(data):
    """tree_probs / q to 8 decimals (float32 values: exact to their precision) for a compact file."""
    for v in data.values():
        for pos in v["positions"]:
            for smp in pos["samples"]:
                smp["tree_probs"] = [round(x, 8) for x in smp["tree_probs"]]
                smp["q"] = round(smp["q"], 8)
    return data


def run_part(name, samples, pi, out):
    """One position of a resnet set in its own process (several run side by side on the host's cores;
    `merge` joins the parts): `resnet_single <samples> <position> <out.json>`."""
    gt = {"resnet_single": 1, "resnet_serving": GAME_THREADS, "resnet_eval": 1}[name]
    net, sums = _resnet()
    pos = run_threaded(net, samples, f"{name}[{pi}]", gt, positions=[POSITIONS[pi]], evaluate=name == "resnet_eval")
    json.dump(dict(threads_per_worker=gt, net_checksums=sums, pi=pi, position=pos[0]), open(out, "w"))


def merge(name, parts, append=False):
    """Set `name` in the fixture from the part files: parts of the same position (`pi`) are
    concatenated (each part process seeds numpy from OS entropy, so parts are independent samples)
    and their expansion counts summed.  With `append` the fixture's existing samples of a position
    are kept and the parts' samples added after them (round 5: positions 0-2 grew 1,000 -> 4,000)."""
    data = json.load(open(OUT))
    ps = [json.load(open(f)) for f in parts]
    by_pi = {}
    if append and name in data:
        for pi, pos in enumerate(data[name]["positions"]):
            by_pi[pi] = dict(pos)
    for p in ps:
        pi, pos = p["pi"], p["position"]
        assert pos["opening"] == POSITIONS[pi]
        if pi not in by_pi:
            by_pi[pi] = dict(opening=pos["opening"], samples=[], expansions=0, re_expansions=0)
        cur = by_pi[pi]
        assert cur["opening"] == pos["opening"]
        cur["samples"] = cur["samples"] + pos["samples"]
        cur["expansions"] += pos["expansions"]
        cur["re_expansions"] += pos["re_expansions"]
    if name == "resnet_eval":  # a subset of the positions: each entry keeps its POSITIONS index
        for pi, cur in by_pi.items():
            cur["pi"] = pi
    else:
        assert sorted(by_pi) == list(range(len(by_pi))), sorted(by_pi)
    data[name] = dict(sims=SIMS, thread_count=THREADS, game="connect4", threads_per_worker=ps[0]["threads_per_worker"],
                      evaluate=name == "resnet_eval",
                      net="ResidualTower(7,6,7,num_blocks=20,filter_factor=32) seed 0",
                      net_checksums=ps[0]["net_checksums"], positions=[by_pi[i] for i in sorted(by_pi)])
    json.dump(_rounded(data), open(OUT, "w"), separators=(",", ":"))


def main():
    torch.multiprocessing.set_start_method("spawn")  # as the reference's entry points (main.py:109)
    os.chdir("/tmp")  # reference modules may write logs into cwd
    os.makedirs("/tmp/g6_saves", exist_ok=True)
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("merge", "merge_append"):  # merge[_append] <set> <part0.json> <part1.json> ...
        return merge(sys.argv[2], sys.argv[3:], append=which == "merge_append")
    if len(sys.argv) == 5:  # <set> <samples> <position> <out.json>
        return run_part(which, int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
    data = json.load(open(OUT)) if os.path.exists(OUT) else {}
    common = dict(sims=SIMS, thread_count=THREADS, game="connect4")
    np.random.seed(6)
    rn = "ResidualTower(7,6,7,num_blocks=20,filter_factor=32) seed 0"
    for name, gt in (("serving", GAME_THREADS), ("single", 1)):
        # serving: threads_per_worker game threads share one worker's queue pool, the
        # reference's default deployment; single: one game thread (its 4 search threads only)
        if which in ("table", "table_" + name, "all"):
            torch.set_num_threads(2)
            data["table_" + name] = dict(common, threads_per_worker=gt, net="table", salt=TABLE_SALT,
                                         positions=run_threaded(TableNetModule(7, TABLE_SALT), 400,
                                                                "table_" + name, gt))
            json.dump(_rounded(data), open(OUT, "w"), separators=(",", ":"))
        if which in ("resnet", "resnet_" + name, "all"):
            torch.set_num_threads(6)
            net, sums = _resnet()
            data["resnet_" + name] = dict(common, threads_per_worker=gt, net=rn, net_checksums=sums,
                                          positions=run_threaded(net, 160, "resnet_" + name, gt))
            json.dump(_rounded(data), open(OUT, "w"), separators=(",", ":"))
    if which in ("resnet_seq", "all"):
        _, sums = _resnet()
        data["resnet_seq"] = dict(common, thread_count=1, threads_per_worker=1, net=rn, net_checksums=sums,
                                  positions=run_sequential(160))
        json.dump(_rounded(data), open(OUT, "w"), separators=(",", ":"))
    print("done")


if __name__ == "__main__":
    main()
