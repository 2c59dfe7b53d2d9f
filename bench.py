#!/usr/bin/env python3
"""Self-play positions/sec — Connect4 7x6, 200 sims/move, 4096 concurrent games per GPU.

BASELINE.json metric "self-play positions/sec (Connect4, 200 sims/move) at
1/2/4/8 MI355X" on configs[1]: ResNet-128 (ResidualTower filter_factor=32,
num_blocks=20, random init, torch.manual_seed(0)), fp16 leaf evaluation (the reference's
autocast inference dtype; --dtype bf16 for the bf16 trunk, reported as secondary_dtype by default).

A *step* is one ply of every game slot of every rank: 200 PUCT simulations
(select -> ResNet -> expand/backup) per game, then the move, Move records,
env step and tree reuse (engine.SelfPlayEngine.ply).  Finished games are
refilled immediately (steady state); finished games' Move records are staged
on each rank's device and, once per episode batch (--exchange-every plies), the
episode statistics are all-reduced and the records gathered to rank 0 (the
replay owner), as in the north star.  Each GPU's games are held in
--lanes arenas (default 2, engine.LanedEngine) on their own HIP streams, so one
arena's tree kernels run beside the other's ResNet launch.  Pending leaves of a
simulation step that are the same network input share one evaluation (batch
leaf dedup, default; --no-leaf-dedup evaluates every leaf in its own row as the
reference's InferenceWorker does): the searches are bit-identical either way
(tests/test_gpu_engine.py), and the line reports nn.rows beside nn.leaves.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       torchrun --nproc-per-node N bench.py --gpus N ...
Prints ONE JSON line on rank 0.  Without torchrun, --gpus N > 1 starts the N rank processes itself
(before this process touches the GPU) with torchrun's environment, one per GPU; it refuses N ranks
on fewer visible GPUs unless SPMCTS_ALLOW_OVERSUBSCRIBE=1 (a rehearsal; with SPMCTS_DIST_BACKEND=gloo,
since RCCL refuses two ranks on one GPU).

Secondary workloads (BASELINE.json configs; not the headline line):
  --sims 800 --games 16384 --filter-factor 64   config 3 (deep trees, ResNet-256)
  --mode arena --games 8192                     config 5: arena evaluation, two frozen nets
                                                (seeds 0 / 1), evaluate mode, no Move records;
                                                metric = games finished per second
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

TRAFFIC_FILE = os.path.join(HERE, "profiles", "r01_bench_prof", "k_tower_traffic.json")  # --search-threads 1
TRAFFIC_FILE_K4 = os.path.join(HERE, "profiles", "r06_bench_prof", "k_tower_traffic.json")  # 4 (default)
TREE_TRAFFIC_FILE_K4 = os.path.join(HERE, "profiles", "r06_tree_pmc", "tree_traffic.json")
# in-bench MFMA-busy share (and profiled clock) of the timed k_tower_dyn dispatches (one PMC pass per trunk dtype,
# scripts/gpu_r06a.sh -> scripts/tower_util.py): the roofline's frac ~ busy x clock / 2.4 GHz / 0.833
CLOCK_FILES = {"fp16": os.path.join(HERE, "profiles", "r06_bench_prof", "tower_util_bench_fp16.json"),
               "bf16": os.path.join(HERE, "profiles", "r05_bench_prof", "tower_util_bench_bf16.json")}

# MI355X reference figures (/opt/skills/guides/MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0
BF16_DENSE_PEAK_TFLOPS = 2500.0


def resnet_flops_per_leaf(W, H, A, filter_factor, num_blocks):
    """Dense FLOPs (2 x MAC) of one ResidualTower forward (games/general/modules.py:88-107)."""
    C, ff, cells = 4 * filter_factor, filter_factor, W * H
    conv3 = 2 * 9 * C * C * cells
    f = 2 * 9 * 3 * C * cells + 2 * num_blocks * conv3
    f += 2 * (2 * C * ff * cells)  # two 1x1 head convs
    f += 2 * ff * cells * A + 2 * ff * cells * 8 * ff + 2 * 8 * ff
    return f


def executed_trunk_flops_per_leaf(W, H, filter_factor, num_blocks):
    """MFMA FLOPs the fused trunk ISSUES per board (C4 edge-tile layout, csrc/tower_edge.h): every conv3x3
    of the residual blocks skips the 12 of 72 (cell tile, tap) pairs whose taps read zero padding only
    (5/6 of the dense MFMAs run); the stem (3 input planes, all 9 taps) and the 1x1 head convs run dense.
    (A batch's one partly empty tail tile issues MFMAs for its empty board slots too; they are not counted.)"""
    C, ff, cells = 4 * filter_factor, filter_factor, W * H
    return 2 * 9 * 3 * C * cells + 2 * num_blocks * (2 * 9 * C * C * cells) * 5 / 6 + 2 * (2 * C * ff * cells)


class GfxClock:
    """The GPU's graphics clock over the timed region, measured in THIS run: a background thread reads
    amdsmi's gpu_metrics (current_gfxclks of the XCDs, MHz) every `period` seconds between start() and
    stop() and reports their mean.  The timed region is >= 95 % trunk dispatches, so the mean is the clock
    the trunk ran at; the roofline's frac_at_clock = achieved / (peak x clock / 2.4 GHz)."""

    def __init__(self, device, period=0.01):
        import threading

        self.samples, self.err, self.period = [], None, period
        self._stop = threading.Event()
        self._thread = None
        try:
            import amdsmi
            import torch

            amdsmi.amdsmi_init()
            self._smi = amdsmi
            pr = torch.cuda.get_device_properties(device)
            bdf = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0"
            self.bdf = bdf
            self._h = amdsmi.amdsmi_get_processor_handle_from_bdf(bdf)
            self._read()  # fail here, not in the thread
        except Exception as e:  # report the reason in the line; the bench still runs
            self.err = f"{type(e).__name__}: {e}"

    def _read(self):
        m = self._smi.amdsmi_get_gpu_metrics_info(self._h)
        clks = m.get("current_gfxclks")
        vals = [c for c in (clks if isinstance(clks, (list, tuple)) else []) if isinstance(c, (int, float)) and 0 < c < 65535]
        if not vals and isinstance(m.get("current_gfxclk"), (int, float)):
            vals = [m["current_gfxclk"]]
        act = m.get("gfx_activity")
        return (sum(vals) / len(vals) if vals else None), (act if isinstance(act, (int, float)) and act <= 100 else None)

    def _run(self):
        while not self._stop.is_set():
            try:
                self.samples.append(self._read())
            except Exception as e:
                self.err = f"{type(e).__name__}: {e}"
                return
            self._stop.wait(self.period)

    def start(self):
        import threading

        if self.err is None:
            self._thread = threading.Thread(target=self._run, daemon=True)
            self._thread.start()

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join()
        if self.err is None:
            try:
                self._smi.amdsmi_shut_down()
            except Exception:
                pass

    def report(self):
        clk = [c for c, _ in self.samples if c is not None]
        act = [a for _, a in self.samples if a is not None]
        if not clk:
            return {"clock_ghz": None, "error": self.err or "no gfx clock samples"}
        return {"clock_ghz": sum(clk) / len(clk) / 1e3, "clock_ghz_min": min(clk) / 1e3, "clock_ghz_max": max(clk) / 1e3,
                "samples": len(clk), "gfx_activity_pct": sum(act) / len(act) if act else None,
                "source": f"amdsmi gpu_metrics current_gfxclks (mean over the XCDs), every {self.period * 1e3:.0f} ms "
                          f"over this run's timed region, device {self.bdf}"}


def head_linear_flops(W, H, A, filter_factor):
    ff, cells = filter_factor, W * H
    return 2 * ff * cells * A + 2 * ff * cells * 8 * ff + 2 * 8 * ff


def select_bytes(sims, levels, A=7, threads=1):
    """Algorithmic HBM bytes moved by k_select.

    Per scored level: the child block (A x {n i32, w f64, p f32, child i32}) + vmask = 20A + 4
    (the next level's child-block index comes with the block).  Per simulation: tree header
    (active id, root id/board/player, noise flag, A noise doubles, root n/w/child index) +
    Philox state load/store = 90 + 8A + 128, leaf record writes (16 per path entry + 38).
    k_select_vl (threads > 1) also reads the children's virtual loss (4A) and writes the node's
    (4) per level, and the leaf's lock (4) per sim; its path record is 4 per entry, not 16.
    """
    per_level = 20 * A + 4 + 16 if threads <= 1 else 24 * A + 4 + 4 + 4
    per_sim = 90 + 8 * A + 128 + 38 + (4 if threads > 1 else 0)
    return levels * per_level + sims * per_sim


def expand_bytes(nn_leaves, path_nodes, A=7, threads=1):
    """Algorithmic HBM bytes of the backups in k_expand / k_expand_vl (block init +
    path read-modify-write), per network leaf: its outputs (4A + 4), the new child block (A x {n i32,
    w f64, p f32, child i32, dtype u8, vl i32} = 25A, + valid mask 4), the leaf's own n/w RMW and
    child index (28), the slot record (node ids, boards, mover, row: 30) and the tree's block
    counter + counters (24); per path node n, w and vl read-modify-write + its id (36 with virtual
    loss, 28 without: n/w only).  The refill selects the rolling schedule runs inside k_expand_vl are
    counted by select_bytes."""
    per_leaf = 4 * A + 4 + 25 * A + 4 + 28 + 30 + 24
    per_path = 36 if threads > 1 else 28
    return nn_leaves * per_leaf + path_nodes * per_path


def _random_opening(rng, max_len=16):
    """A non-terminal Connect4 position after 0..max_len uniformly random legal moves (the worker's
    next game starts there), so a short sample covers the mid-game positions a steady-state
    self-play run searches, not only openings."""
    from oracle.envs import Connect4Env

    while True:
        env, acts, player = Connect4Env(), [], 1
        ok = True
        for _ in range(rng.randint(0, max_len)):
            legal = [a for a in range(7) if env.valid_moves()[a]]
            a = legal[rng.randint(len(legal))]
            _, _, done, _ = env.step(a, player)
            if done:
                ok = False
                break
            acts.append(a)
            player = -player
        if ok:
            return acts


def _cpu_worker(args):
    """One host process: the oracle's search (the reference's MCTreeSearch algorithm, numpy RNG) +
    the reference-architecture ResNet in fp32 torch on ONE thread, complete moves only, for
    `seconds`.  Games start at random mid-game positions (`openings`) or from the empty board."""
    seconds, seed, sims, filter_factor, num_blocks, threads, openings = args
    import numpy as np
    import torch

    from oracle.envs import Connect4Env
    from oracle.mcts import NumpyRNG, OracleTree
    from self_play_reinforcement_learning_amd.modules import ResidualTower

    torch.set_num_threads(1)
    torch.manual_seed(0)
    net = ResidualTower(7, 6, 7, num_blocks=num_blocks, filter_factor=filter_factor).eval()
    np.random.seed(seed)
    rng = np.random.RandomState(seed + 1)
    moves = 0

    def new_game():
        tree, env, player = OracleTree("connect4", net, NumpyRNG(), sims, threads=threads), Connect4Env(), 1
        for a in (_random_opening(rng) if openings else []):  # play_action flips the root's player
            tree.play_action(a)
            env.step(a, player)
            player = -player
        return tree, env, player

    with torch.no_grad():
        tree, env, player = new_game()
        t0 = time.time()
        while time.time() - t0 < seconds:
            a = tree.move()
            tree.play_action(a)
            _, _, done, _ = env.step(a, player)
            moves += 1
            player = -player
            if done:
                tree, env, player = new_game()
        dt = time.time() - t0
    return moves, dt


def cpu_baseline(seconds, cores, sims, filter_factor, num_blocks, threads=1, openings=True):
    """The reference's CPU self-play structure restated: `cores` independent play processes (the
    reference runs one SelfPlayWorker per core, self_play_parallel.py:95-171), each running the
    oracle's search with a 1-thread fp32 ResNet, for about `seconds`; positions/s summed over
    processes.  (No IPC inference batching: the reference's proxy adds queue round trips.)
    threads > 1: the oracle's threaded (virtual-loss, rolling) search, same per-leaf network calls.
    openings: games start after 0..16 random moves (mid-game positions, where terminal leaves
    occur), else from the empty board."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    with ctx.Pool(cores) as pool:
        res = pool.map(_cpu_worker, [(seconds, 1000 + i, sims, filter_factor, num_blocks, threads, openings)
                                     for i in range(cores)])
    moves = sum(m for m, _ in res)
    rate = sum(m / dt for m, dt in res)
    out = dict(value=rate, unit="positions/s", cores=cores, kind="port",
               sample=f"{cores} processes x (oracle MCTS, {sims} sims/move, "
                      f"{'sequential' if threads <= 1 else f'{threads} sims in flight (virtual loss)'}, numpy RNG + ResNet-"
                      f"{4 * filter_factor}x{num_blocks} fp32 torch, 1 thread), Connect4 games "
                      f"{'from random 0-16-move openings' if openings else 'from the empty board'}, "
                      f"{moves} complete moves in ~{seconds:.0f} s")
    cal = os.path.join(HERE, "profiles", "r02", "cpu_calibration.json")
    if os.path.exists(cal):
        with open(cal) as f:
            c = json.load(f)
        # the reference's own pipeline over the port run the same way (random openings <-> bench mode), both
        # on the build container's cores, back to back, as positions/s PER CORE: the reference used all
        # c["cores"] cores (c["reference"]["play_workers"] play processes + its InferenceWorker), the port one
        # process per core, so the ratio of per-core rates maps the port's per-core rate on this host to the
        # reference's.  It applies to the same sims in flight per tree (the reference's thread_count).
        port = c["port_bench_mode"] if openings and "port_bench_mode" in c else c["port"]
        ref_pc = c["reference"]["value"] / c["reference"]["cores"]
        port_pc = port["value"] / port["cores"]
        r = ref_pc / port_pc
        # the calibration ran the headline workload (200 sims, ResNet-128x20) at the reference's thread_count
        same_k = threads == c["reference"]["thread_count"] and (sims, filter_factor, num_blocks) == (200, 32, 20)
        out["calibration"] = dict(
            ratio_reference_over_port_per_core=r, source=os.path.relpath(cal, HERE),
            reference_per_core=ref_pc, port_per_core_calibration=port_pc, port_per_core_here=rate / cores,
            calibrated_on=dict(cores=c["cores"], host=c.get("host"), port_sample=port["sample"],
                               reference_sample=f"{c['reference']['play_workers']} play workers x "
                                                f"{c['reference']['threads_per_worker']} game threads x "
                                                f"thread_count {c['reference']['thread_count']} + InferenceWorker"),
            reference_equivalent=rate * r if same_k else None,
            reference_equivalent_per_core=rate / cores * r if same_k else None,
            note=("reference_equivalent = value x the per-core ratio (the reference's multiprocess pipeline vs this "
                  f"port, timed back to back on the build container's {c['cores']} cores), i.e. the reference's "
                  f"pipeline on the {cores} cores used here at the same per-core scaling" if same_k else
                  "not applied: the calibration ran 200 sims, ResNet-128x20, "
                  f"{c['reference']['thread_count']} sims in flight per tree"))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=24, help="timed plies")
    ap.add_argument("--warmup", type=int, default=24,
                    help="untimed plies (24 ~ one game generation: games have reached their steady mix of lengths)")
    ap.add_argument("--games", type=int, default=4096, help="concurrent games per GPU")
    ap.add_argument("--sims", type=int, default=200)
    ap.add_argument("--filter-factor", type=int, default=32)
    ap.add_argument("--blocks", type=int, default=20)
    ap.add_argument("--bucket", type=int, default=256)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true", help="skip the rank-0 Move gather")
    ap.add_argument("--exchange-every", type=int, default=8,
                    help="plies per episode-batch exchange round (Move rows to rank 0 + stats all-reduce)")
    ap.add_argument("--mode", choices=["selfplay", "arena"], default="selfplay")
    ap.add_argument("--no-leaf-dedup", action="store_true",
                    help="evaluate every pending leaf in its own row (default: one row per distinct position "
                         "of a simulation step, include/spmcts.h spmcts_set_leaf_dedup)")
    ap.add_argument("--lanes", type=int, default=2,
                    help="arenas per GPU on their own HIP streams (engine.LanedEngine); 1 = one arena")
    ap.add_argument("--blocks-per-tree", type=int, default=0,
                    help="node blocks per tree; below the worst case the arena recycles subtrees (k_compact)")
    ap.add_argument("--stagger", action="store_true",
                    help="lane i runs i * S / lanes simulation steps behind lane 0 (engine.LanedEngine stagger) "
                         "instead of the lanes in lock step")
    ap.add_argument("--no-cross-dedup", action="store_true",
                    help="lanes > 1: per-lane leaf dedup only (default: a lane-1 leaf whose input lane 0 evaluates in "
                         "the same simulation step takes lane 0's row, engine.LanedEngine cross_dedup)")
    ap.add_argument("--lane0-share", type=float, default=None,
                    help="lanes = 2: lane 0's share of the games.  Default: 0.48 with cross-lane dedup (lane 1, whose "
                         "leaves lane 0 also evaluates, then gets 2,130 of 4,096 games: the lanes' rows balance; measured "
                         "+0.5 %% vs an even split, -0.9 %% at 0.46, profiles/r06/final_bundle/), else an even split")
    ap.add_argument("--no-pack", action="store_true",
                    help="lanes > 1: keep round-aligned tower tiles (no SPMCTS_TOWER_PACK)")
    ap.add_argument("--twin-no-dedup", type=int, default=5, metavar="PLIES",
                    help="after the timed region, turn leaf dedup off and time PLIES more plies of the same games "
                         "(every leaf its own row, as the reference): reported as no_dedup_twin")
    ap.add_argument("--eval-cache", type=int, default=1, metavar="PLIES",
                    help="evaluation cache window (include/spmcts.h spmcts_set_eval_cache): a position evaluated in "
                         "the last PLIES plies takes the cached outputs instead of a network row; 1 (default) = "
                         "within the ply, so every output a timed ply uses was computed in that ply; 0 = off")
    ap.add_argument("--twin-no-cache", type=int, default=5, metavar="PLIES",
                    help="with --eval-cache: after the timed region time PLIES more plies with the cache off "
                         "(per-step leaf dedup alone): reported as no_cache_twin")
    ap.add_argument("--no-clock", action="store_true",
                    help="do not sample the gfx clock (amdsmi) during the timed region")
    ap.add_argument("--progress", action="store_true",
                    help="one stderr line per untimed ply (long warm-ups, e.g. config 3 in steady state)")
    ap.add_argument("--dtype", choices=["bf16", "fp16"], default="fp16",
                    help="element type of the fused trunk's weights / activations (fp32 accumulation); fp16 (the "
                         "default) is the reference's own inference dtype (amp.autocast, inference_worker.py:117)")
    ap.add_argument("--secondary", action="store_true",
                    help="also time the other trunk dtype (bf16 <-> fp16) on a fresh engine with the same seeds, "
                         "--warmup and --steps, reported as secondary_dtype.  Off by default: the headline runs the "
                         "reference's inference dtype (fp16) alone; bf16's search shift is bounded at 0.02 "
                         "(tests/test_gpu_statistical.py SHIFT_TOL), eight times fp16's error")
    ap.add_argument("--no-secondary", dest="secondary", action="store_false", help=argparse.SUPPRESS)
    ap.add_argument("--search-threads", type=int, default=4,
                    help="sims in flight per tree with virtual loss: the reference's thread_count search "
                         "(mcts.py:328-331), 4 in its headline self-play setup (InferenceProxy workers, "
                         "SURVEY §6); 1 = sequential search (bit-exact to the reference's sequential fixtures)")
    args = ap.parse_args()
    arena_mode = args.mode == "arena"

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU, started here (the driver's `python bench.py --gpus N` form); the ranks
        # get torchrun's environment and this process never touches the GPU
        from self_play_reinforcement_learning_amd import distributed as D

        try:
            D.check_devices(args.gpus)
        except RuntimeError as e:
            print(f"bench.py: {e}", file=sys.stderr, flush=True)
            sys.exit(2)
        sys.exit(D.launch_script([os.path.abspath(__file__)] + sys.argv[1:], args.gpus))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}; the launched ranks count",
              file=sys.stderr, flush=True)

    # The CPU baseline runs FIRST, in child processes started before this process touches the GPU
    # (children of a GPU-initialised process must not exec); rank 0 of a 1-process run only.
    env_rank, env_world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    cpu = None
    if env_rank == 0 and env_world == 1 and not args.no_cpu_baseline and not arena_mode:
        cpu = cpu_baseline(args.cpu_seconds, min(16, os.cpu_count() or 1), args.sims, args.filter_factor, args.blocks,
                           threads=args.search_threads)

    import torch

    from self_play_reinforcement_learning_amd import distributed as D
    from self_play_reinforcement_learning_amd.engine import LanedEngine, SelfPlayEngine, union_ms
    from self_play_reinforcement_learning_amd.modules import ResidualTower

    rank, world, local = D.init_from_env()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    torch.manual_seed(0)
    net = ResidualTower(7, 6, 7, num_blocks=args.blocks, filter_factor=args.filter_factor).to(dev).eval()
    opponent = None
    if arena_mode:  # BASELINE config 5: two frozen nets, greedy (evaluate-mode) MCTS on both sides
        torch.manual_seed(1)
        opponent = ResidualTower(7, 6, 7, num_blocks=args.blocks, filter_factor=args.filter_factor).to(dev).eval()
    tdt = {"bf16": torch.bfloat16, "fp16": torch.float16}[args.dtype]
    kw = dict(iterations=args.sims, seed=1234 + rank, device=dev, bucket=args.bucket, opponent=opponent, dtype=tdt,
              evaluate=arena_mode, record=not arena_mode, search_threads=args.search_threads,
              blocks_per_tree=args.blocks_per_tree, leaf_dedup=False if args.no_leaf_dedup else None,
              eval_cache=0 if (args.no_leaf_dedup or args.search_threads < 2) else args.eval_cache)
    if args.lanes > 1:
        lane_sizes = None
        share = args.lane0_share
        if share is None and not args.no_cross_dedup and not arena_mode and args.search_threads > 1 \
                and not args.no_leaf_dedup and not args.stagger:
            share = 0.48  # cross-lane dedup will pair the lanes (LanedEngine cross_dedup)
        if share is not None and args.lanes == 2:
            n0 = int(round(args.games * share))
            lane_sizes = [n0, args.games - n0]
        eng = LanedEngine("connect4", net, n_games=args.games, lanes=args.lanes, pack=not args.no_pack,
                          stagger=args.stagger, cross_dedup=False if args.no_cross_dedup else None,
                          lane_sizes=lane_sizes, **kw)
    else:
        eng = SelfPlayEngine("connect4", net, n_games=args.games, **kw)
    gathered = []
    # finished games' Move rows: staged on each rank's device, gathered to rank 0 once per episode
    # batch (every --exchange-every plies, and once more at the end of the timed region) together
    # with the episode statistics (distributed.MoveExchange); a single process hands them on at once
    ex = D.MoveExchange(42, 7, sink=lambda g: gathered.append(int(g["z"].shape[0])), every=args.exchange_every)

    def one_step():
        eng.ply(on_moves=ex.stage if not (args.no_gather or arena_mode) else None)
        # statistics are read (a host sync on the device counters) only for a real exchange round
        ex.end_ply(eng.stats_vector if D.is_distributed() else None)

    tw = time.perf_counter()
    for i in range(args.warmup):
        one_step()
        if args.progress and rank == 0:
            print(f"bench.py: warm-up ply {i + 1}/{args.warmup} at {time.perf_counter() - tw:.1f} s", file=sys.stderr,
                  flush=True)
    if D.is_distributed() and args.warmup % args.exchange_every:
        ex.end_ply(eng.stats_vector, force=True)
    ex._plies = ex.rounds = ex.rows_gathered = 0  # the timed region starts a fresh episode batch
    ex.seconds = 0.0
    eng.check()
    c0 = eng.counters()
    eng.enable_timers(True)

    gclk = None if args.no_clock else GfxClock(dev)
    D.barrier()
    torch.cuda.synchronize()
    ref = torch.cuda.Event(enable_timing=True)  # time origin of the launch intervals (all lanes' streams)
    ref.record()
    if gclk is not None:
        gclk.start()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_step()
    if D.is_distributed() and args.steps % args.exchange_every:
        ex.end_ply(eng.stats_vector, force=True)  # the rows of the last partial batch reach rank 0 too
    D.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if gclk is not None:
        gclk.stop()
    elapsed_max = D.all_reduce_max(elapsed)

    c1 = eng.counters()
    eng.check()
    moves_local = c1["moves"] - c0["moves"]
    # per-rank lines (an all_gather on every rank): stragglers and exchange cost show in a scaling record
    per_rank = D.rank_report([moves_local / elapsed if elapsed else 0.0, elapsed, ex.rounds,
                              ex.seconds / max(1, ex.rounds) * 1e3, ex.rows_gathered])
    tot = D.all_reduce_stats([moves_local, c1["sims"] - c0["sims"], c1["games_finished"] - c0["games_finished"]])
    moves_all, sims_all, games_all = (int(x) for x in tot)

    # ---- tree kernels (HIP events around k_select* / k_expand* on each lane's stream).  With K > 1
    # the rolling schedule runs most selects inside k_expand_vl (each slot refilled right after its
    # backup), so the two kernels are reported together: algorithmic bytes of every select level and
    # every backup / block init over their summed durations.  With two lanes a tree kernel of one lane
    # shares the chip with the other lane's tower dispatch, so these durations include that wait.
    sel_ms = eng.select_timer.total_ms()
    exp_ms = eng.expand_timer.total_ms()
    sel_launches = eng.select_timer.count()
    exp_launches = eng.expand_timer.count()
    sims_local = c1["sims"] - c0["sims"]
    levels_local = c1["depth_sum"] - c0["depth_sum"]
    nn_local = c1["nn_leaves"] - c0["nn_leaves"]
    path_nodes = levels_local * (nn_local / max(1, sims_local))
    tree_bytes = select_bytes(sims_local, levels_local, threads=args.search_threads) + \
        expand_bytes(nn_local, path_nodes, threads=args.search_threads)
    tree_dispatches = sel_launches + exp_launches
    tree_s = (sel_ms + exp_ms) / 1e3
    bytes_per_launch = tree_bytes / max(1, tree_dispatches)
    sel_avg_s = tree_s / max(1, tree_dispatches)
    achieved = tree_bytes / tree_s / 1e9 if tree_s > 0 else 0.0
    tree_traffic, tree_traffic_src = None, None
    tfile = TREE_TRAFFIC_FILE_K4 if args.search_threads > 1 else None
    if tfile and os.path.exists(tfile) and (args.games, args.sims, args.filter_factor, args.blocks) == (4096, 200, 32, 20):
        with open(tfile) as f:
            tree_traffic = json.load(f)["bytes_per_dispatch"]
        tree_traffic_src = os.path.relpath(tfile, HERE)

    # ---- network (MFMA) share: busy time = union of the network launches of all lanes
    nn_ms = union_ms(eng.nn_timer.intervals(ref))
    # rows the network actually evaluated (with leaf dedup, one per distinct position of a step)
    rows = c1["nn_rows"] - c0["nn_rows"]
    leaves = c1["nn_leaves"] - c0["nn_leaves"]
    fpl = resnet_flops_per_leaf(7, 6, 7, args.filter_factor, args.blocks)
    nn_tflops = rows * fpl / (nn_ms / 1e3) / 1e12 if nn_ms > 0 else 0.0
    # ---- dominant kernel: k_tower (HIP events around each tower dispatch on its lane's stream).
    # With L lanes the L dispatches of one simulation step run concurrently on the chip, so a
    # "launch" here is that group of L dispatches and its duration is their busy (union) time; at
    # L = 1 this is exactly the per-dispatch average.  The per-dispatch average (what rocprof's
    # kernel stats report) is kept beside it as avg_dispatch_us.
    tw = eng.tower_timer
    tw_dispatches = tw.count() if tw is not None else 0
    tw_sum_ms = tw.total_ms() if tw_dispatches else 0.0
    tw_ms = union_ms(tw.intervals(ref)) if tw_dispatches else 0.0
    lanes = max(1, args.lanes)
    tw_launches = tw_dispatches // lanes
    trunk_fpl = fpl - head_linear_flops(7, 6, 7, args.filter_factor)
    tw_flops_per_launch = rows * trunk_fpl / max(1, tw_launches)
    tw_avg_s = tw_ms / 1e3 / max(1, tw_launches)
    tw_tflops = tw_flops_per_launch / tw_avg_s / 1e12 if tw_avg_s > 0 else 0.0
    # PMC-measured traffic of the same kernel on the same bench command (rocprofv3 FETCH_SIZE /
    # WRITE_SIZE passes, scripts/gpu_prof_bench.sh -> scripts/pmc_traffic.py); bench.py cannot run
    # the profiler itself, so it reports the committed measurement for the default workload
    traffic, traffic_src = None, None
    tfile = {1: TRAFFIC_FILE, 4: TRAFFIC_FILE_K4}.get(args.search_threads)
    if tfile and os.path.exists(tfile) and (args.games, args.sims, args.filter_factor, args.blocks) == (4096, 200, 32, 20):
        with open(tfile) as f:
            tj = json.load(f)
        # per-dispatch bytes x dispatches per launch (a launch = one simulation step over all lanes)
        traffic = tj.get("bytes_per_dispatch", tj["bytes_per_launch"]) * max(1, args.lanes)
        traffic_src = os.path.relpath(tfile, HERE)

    # the clock of THIS run's timed region (amdsmi, GfxClock): the peak at that clock and the frac against it
    clock = gclk.report() if gclk is not None else None
    if clock is not None and clock.get("clock_ghz"):
        ghz = clock["clock_ghz"]
        clock.update(peak_at_clock=BF16_DENSE_PEAK_TFLOPS * ghz / 2.4,
                     frac_at_clock=tw_tflops / (BF16_DENSE_PEAK_TFLOPS * ghz / 2.4),
                     note="peak scaled linearly from 2.5 PFLOP/s at 2.4 GHz to the clock this run's timed region held")
    # MFMA busy share of the trunk from the committed in-bench PMC pass (another run of this command: the
    # profiler cannot run inside bench.py), for the factorisation frac ~ busy x clock/2.4 / executed share
    mfma_busy_pmc = None
    cfile = CLOCK_FILES.get(args.dtype)
    if cfile and os.path.exists(cfile) and (args.games, args.sims, args.filter_factor, args.blocks) == (4096, 200, 32, 20):
        with open(cfile) as f:
            cj = json.load(f)
        mfma_busy_pmc = {"mfma_busy_frac": cj["mfma_busy_frac_weighted"], "clock_ghz": cj["clock_ghz_weighted"],
                         "dispatches": cj.get("dispatches"), "source": os.path.relpath(cfile, HERE),
                         "note": "a profiled run of this command (rocprofv3 PMC: SQ_VALU_MFMA_BUSY_CYCLES, "
                                 "GRBM_GUI_ACTIVE), not this run"}
    ex_fpl = executed_trunk_flops_per_leaf(7, 6, args.filter_factor, args.blocks)
    ex_tflops = tw_tflops * ex_fpl / trunk_fpl

    out = {
        "metric": f"self-play positions/sec (Connect4, {args.sims} sims/move)",
        "value": moves_all / elapsed_max,
        "unit": "positions/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed_max / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic (self-generated games, random-init ResNet weights, torch.manual_seed(0))",
        "config": {
            "workload": f"connect4 7x6 self-play, {args.sims} sims/move, {args.games} concurrent games per GPU "
                        f"(2 trees each), ResNet-{4 * args.filter_factor}x{args.blocks} {args.dtype} leaf eval, fp64 tree stats",
            "games_per_gpu": args.games,
            "global_games": args.games * world,
            "sims_per_move": args.sims,
            "net": f"ResidualTower(filter_factor={args.filter_factor}, num_blocks={args.blocks})",
            "parallelism": f"dp{world}",
            "lanes_per_gpu": max(1, args.lanes),
            "lanes_staggered": bool(getattr(eng, "stagger", False)) if args.lanes > 1 else False,
            "lane_games": [e.n_games for e in eng.lanes] if args.lanes > 1 else [args.games],
            "search_threads": args.search_threads,
            "leaf_dedup": bool(getattr(eng, "leaf_dedup", False)),
            "cross_lane_dedup": bool(getattr(eng, "cross_dedup", False)),
            "eval_cache_plies": int(getattr(eng, "eval_cache", 0)),
            "eval_cache_note": ("a leaf whose network input was evaluated earlier in the same ply takes those outputs "
                                "(one evaluation per distinct input per ply; nothing computed before a ply is reused "
                                "in it); the searches are bit-identical to the cache-off run "
                                "(tests/test_gpu_engine.py::test_eval_cache_is_exact); no_cache_twin times the plies "
                                "after the timed region with it off") if getattr(eng, "eval_cache", 0) == 1 else None,
        },
        "roofline": {
            "kernel": f"tower::k_tower_dyn (fused ResNet-{4 * args.filter_factor}x{args.blocks} trunk, {args.dtype} MFMA)",
            "bound": "mfma",
            "achieved": tw_tflops,
            "peak": BF16_DENSE_PEAK_TFLOPS,
            "unit": "TFLOP/s",
            "frac": tw_tflops / BF16_DENSE_PEAK_TFLOPS,
            "traffic": traffic,
            "traffic_unit": "bytes/launch (L2<->fabric, PMC)",
            "traffic_source": traffic_src,
            "flops_per_launch": tw_flops_per_launch,
            "flops_per_leaf": trunk_fpl,
            "rows_per_launch": rows / max(1, tw_launches),
            "avg_launch_us": tw_avg_s * 1e6,
            "launches": tw_launches,
            "lanes": lanes,
            "launch_def": (f"one simulation step = {lanes} concurrent k_tower_dyn dispatches (one per lane stream); "
                           "duration = their union busy time" if lanes > 1 else "one k_tower_dyn dispatch"),
            "avg_dispatch_us": tw_sum_ms / max(1, tw_dispatches) * 1e3,
            "dispatches": tw_dispatches,
            "executed": {"achieved": ex_tflops, "frac": ex_tflops / BF16_DENSE_PEAK_TFLOPS,
                         "flops_per_leaf": ex_fpl,
                         "note": "MFMA FLOPs the trunk issues (the edge tiles skip the 1/6 of the block convs' "
                                 "dense MFMAs that multiply zero padding only), same launches and time"},
            "clock": clock,
            "mfma_busy_pmc": mfma_busy_pmc,
        },
        "tree_roofline": {
            "kernel": ("k_select<C4> + k_expand<C4> (PUCT tree walk, backup)" if args.search_threads <= 1 else
                       f"k_select_vl<C4> + k_expand_vl<C4> (rolling search, {args.search_threads} sims in flight per "
                       f"tree: walks, backups, refills)"),
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": tree_traffic,
            "traffic_unit": "bytes/dispatch (L2<->fabric, PMC, both kernels)",
            "traffic_source": tree_traffic_src,
            "bytes_per_launch": bytes_per_launch,
            "avg_launch_us": sel_avg_s * 1e6,
            "launches": tree_dispatches,
            "select": {"dispatches": sel_launches, "ms": sel_ms},
            "expand": {"dispatches": exp_launches, "ms": exp_ms},
            "note": "durations co-scheduled with the other lane's tower dispatch" if args.lanes > 1 else None,
        },
        "nn": {
            "bound": "mfma",
            "achieved_tflops": nn_tflops,
            "peak_tflops": BF16_DENSE_PEAK_TFLOPS,
            "frac": nn_tflops / BF16_DENSE_PEAK_TFLOPS,
            "flops_per_leaf": fpl,
            "rows": rows,
            "leaves": leaves,
            "leaf_dedup": bool(getattr(eng, "leaf_dedup", False)),
            "rows_per_leaf": rows / max(1, leaves),
            "cache_rows": c1["cache_rows"] - c0["cache_rows"],
            "nn_ms": nn_ms,
            "share_of_step": nn_ms / 1e3 / elapsed if elapsed else None,
        },
        "ranks": {
            "world_size": torch.distributed.get_world_size() if D.is_distributed() else 1,
            "backend": torch.distributed.get_backend() if D.is_distributed() else None,
            "positions_per_s_min": min(r[0] for r in per_rank),
            "positions_per_s_max": max(r[0] for r in per_rank),
            "per_rank": [{"rank": i, "positions_per_s": r[0], "timed_s": r[1], "exchange_rounds": int(r[2]),
                          "exchange_ms_per_round": r[3], "rows_received": int(r[4])} for i, r in enumerate(per_rank)],
        },
        "exchange": {"backend": torch.distributed.get_backend() if D.is_distributed() else None,
                     "every_plies": args.exchange_every, "rounds": ex.rounds, "rows_to_rank0": ex.rows_gathered,
                     "ms_per_round": ex.seconds / max(1, ex.rounds) * 1e3,
                     "share_of_timed_region": ex.seconds / elapsed if elapsed else None},
        "tree": {
            "sims": sims_all,
            "mean_select_levels": levels_local / max(1, sims_local),
            "terminal_leaf_frac": (c1["terminal_leaves"] - c0["terminal_leaves"]) / max(1, sims_local),
            "games_finished": games_all,
            "select_ms_share": sel_ms / 1e3 / elapsed if elapsed else None,
            "expand_ms_share": exp_ms / 1e3 / elapsed if elapsed else None,
            "leaked_sims": c1["leaked_sims"] - c0["leaked_sims"],
            "blocks_in_use_max": c1["blocks_in_use_max"],
            "compactions": c1["compactions"] - c0["compactions"],
        },
        "cpu_baseline": None,
    }
    if arena_mode:
        out["metric"] = f"arena evaluation games/sec (Connect4, {args.sims} sims/move, two frozen nets)"
        out["value"] = games_all / elapsed_max
        out["unit"] = "games/s"
        out["positions_per_s"] = moves_all / elapsed_max
        out["config"]["workload"] = (f"connect4 7x6 arena evaluation, {args.sims} sims/move, {args.games} concurrent "
                                     f"games per GPU, policy ResNet-{4 * args.filter_factor}x{args.blocks} (seed 0) vs "
                                     f"opponent (seed 1), evaluate mode (temp/20, noise on), no Move records")
    out["cpu_baseline"] = cpu

    def twin(plies):
        """`plies` more plies on the same arenas right after the timed region: (the headline's unit per second --
        positions/s, games/s in arena mode --, ms per ply, rows per leaf)."""
        eng.check()
        t_c0 = eng.counters()
        D.barrier()
        torch.cuda.synchronize()
        t_t0 = time.perf_counter()
        for _ in range(plies):
            one_step()
        if D.is_distributed() and plies % args.exchange_every:
            ex.end_ply(eng.stats_vector, force=True)
        D.barrier()
        torch.cuda.synchronize()
        t_el = D.all_reduce_max(time.perf_counter() - t_t0)
        t_c1 = eng.counters()
        eng.check()
        unit = "games_finished" if arena_mode else "moves"
        t_moves = int(D.all_reduce_stats([t_c1[unit] - t_c0[unit]])[0])
        return (t_moves / t_el, t_el / plies * 1e3,
                (t_c1["nn_rows"] - t_c0["nn_rows"]) / max(1, t_c1["nn_leaves"] - t_c0["nn_leaves"]))

    if args.twin_no_cache > 0 and getattr(eng, "eval_cache", 0):
        for e in getattr(eng, "lanes", [eng]):
            e.arena.set_eval_cache(0)
            e.eval_cache = 0
        v_, ms_, rpl_ = twin(args.twin_no_cache)
        out["no_cache_twin"] = {
            "plies": args.twin_no_cache, "value": v_, "unit": out["unit"], "ms_per_step": ms_, "rows_per_leaf": rpl_,
            "note": "the plies right after the timed region, evaluation cache off (spmcts_set_eval_cache 0): leaf "
                    "dedup within each simulation step only"}
    if args.twin_no_dedup > 0 and getattr(eng, "leaf_dedup", False):
        # the same arenas, right after the timed region: every leaf gets its own network row
        for e in getattr(eng, "lanes", [eng]):
            e.arena.set_leaf_dedup(False)
            e.leaf_dedup = False
        eng.leaf_dedup = False
        v_, ms_, rpl_ = twin(args.twin_no_dedup)
        out["no_dedup_twin"] = {
            "plies": args.twin_no_dedup, "value": v_, "unit": out["unit"], "ms_per_step": ms_, "rows_per_leaf": rpl_,
            "note": "the plies right after the timed region, leaf dedup off (spmcts_set_leaf_dedup): every leaf "
                    "evaluated in its own row, as the reference's InferenceWorker"}
    if args.secondary and not arena_mode:
        # the other trunk element type (bf16 <-> fp16) on a FRESH engine with the same seeds, warm-up and
        # timed plies as the headline (games of the same age, so the two lines compare like for like);
        # `value` is the --dtype line.  The headline arenas are released first.
        other = {"bf16": "fp16", "fp16": "bf16"}[args.dtype]
        for e in getattr(eng, "lanes", [eng]):
            e.arena.close()
        del eng
        torch.cuda.empty_cache()
        kw2 = dict(kw, dtype={"bf16": torch.bfloat16, "fp16": torch.float16}[other])
        if args.lanes > 1:
            eng2 = LanedEngine("connect4", net, n_games=args.games, lanes=args.lanes, pack=not args.no_pack,
                               stagger=args.stagger, cross_dedup=False if args.no_cross_dedup else None,
                               lane_sizes=lane_sizes, **kw2)
        else:
            eng2 = SelfPlayEngine("connect4", net, n_games=args.games, **kw2)
        ex2 = D.MoveExchange(42, 7, sink=lambda g: None, every=args.exchange_every)

        def step2():
            eng2.ply(on_moves=ex2.stage if not args.no_gather else None)
            ex2.end_ply(eng2.stats_vector if D.is_distributed() else None)

        for _ in range(args.warmup):
            step2()
        if D.is_distributed() and args.warmup % args.exchange_every:
            ex2.end_ply(eng2.stats_vector, force=True)
        eng2.check()
        s_c0 = eng2.counters()
        eng2.enable_timers(True)
        D.barrier()
        torch.cuda.synchronize()
        ref2 = torch.cuda.Event(enable_timing=True)
        ref2.record()
        s_t0 = time.perf_counter()
        for _ in range(args.steps):
            step2()
        if D.is_distributed() and args.steps % args.exchange_every:
            ex2.end_ply(eng2.stats_vector, force=True)
        D.barrier()
        torch.cuda.synchronize()
        s_el = D.all_reduce_max(time.perf_counter() - s_t0)
        s_c1 = eng2.counters()
        eng2.check()
        s_moves = int(D.all_reduce_stats([s_c1["moves"] - s_c0["moves"]])[0])
        s_rows = s_c1["nn_rows"] - s_c0["nn_rows"]
        t2 = eng2.tower_timer
        s_launches = max(1, t2.count() // lanes)
        s_tw_s = union_ms(t2.intervals(ref2)) / 1e3 / s_launches
        s_tflops = s_rows * trunk_fpl / s_launches / s_tw_s / 1e12 if s_tw_s > 0 else 0.0
        out["secondary_dtype"] = {
            "dtype": other, "value": s_moves / s_el, "unit": "positions/s", "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": s_el / args.steps * 1e3,
            "rows_per_leaf": s_rows / max(1, s_c1["nn_leaves"] - s_c0["nn_leaves"]),
            "roofline": {"achieved": s_tflops, "peak": BF16_DENSE_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": s_tflops / BF16_DENSE_PEAK_TFLOPS, "avg_launch_us": s_tw_s * 1e6},
            "note": f"a fresh engine with the same seeds, warm-up and timed plies as the headline, the fused trunk "
                    f"and heads in {other}; the headline `value` is --dtype {args.dtype}"}
        for e in getattr(eng2, "lanes", [eng2]):
            e.arena.close()
    if rank == 0:
        print(json.dumps(out), flush=True)
    if D.is_distributed():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
