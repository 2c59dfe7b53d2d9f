"""Oracle restatement of the reference MCTS (games/algos/mcts.py).  TEST INFRASTRUCTURE.

Sequential (single-thread) semantics of MCTreeSearch — the mode the reference
runs whenever its network is not an InferenceProxy (mcts.py:154, :332-334) and
the mode whose results are deterministic under `np.random.seed`.

Restated faithfully, including the quirks the HIP arena must reproduce:
  * virtual loss makes the parent count sqrt(N + 1) while its children are
    scored (mcts.py:345, :76);
  * the leaf is evaluated from the just-moved player's perspective (mcts.py:316);
  * Dirichlet noise covers invalid children too (mcts.py:50-53);
  * terminal leaves never get children and are re-stepped on every visit
    (mcts.py:306-314, :357);
  * the unvisited child reached by play_action is expanded and backed up once
    (mcts.py:201-209);
  * temperature is always 1 in self-play, temp/20 in evaluate mode
    (mcts.py:182-183, :273-274).

Backup (mcts.py:94-98) recurses to the ORIGINAL game root; the nodes above the
active root are never read again, so the restatement stops at the active root
(observationally equivalent).

Threaded mode (`threads=K > 1`, the reference's `thread_count` search when its
network is an InferenceProxy, mcts.py:154, :328-331): each of the reference's K
threads runs select -> network wait -> backup and then takes the next
search_node task, so ~K sims are always in flight and each new select sees the
other K-1 pending (a rolling window).  Its threads interleave
nondeterministically, so the restatement fixes the rolling order: K pending
slots, completed oldest-first (slot order) and each refilled right after its
backup; a sim that ends without a network call (terminal leaf, backed up at
once; or a leak, mcts.py:349-354) frees its slot for the next sim at once.
This is the schedule the HIP arena's k_select_vl / k_expand_vl implement
(bit-exact on shared tapes).  Against the reference itself it is pinned
statistically: G6 (tests/golden/threaded_stats.json) holds root visit
distributions of the reference's own threaded search behind a real
InferenceProxy / InferenceWorker.

RNG: every random draw goes through an `rng` object with the reference's call
order: per search one `dirichlet(alpha, A)`, per descended
level one `rand(A)`, per move one uniform for `np.random.choice`.
`NumpyRNG` draws from numpy's legacy global RandomState exactly as the
reference does; `TapeRNG` replays (and `RecordingRNG` records) the same doubles
as a flat per-tree stream — the form the HIP arena consumes in tape mode.
"""
import math

import numpy as np

from .envs import GameOver, make_env  # noqa: F401


# ---------------------------------------------------------------------------- RNG
class NumpyRNG:
    """numpy legacy global RandomState, same calls as mcts.py:50, :355, :280."""

    def dirichlet(self, alpha, k):
        return np.random.dirichlet([alpha] * k)

    def rand(self, k):
        return np.random.rand(k)

    def choice_index(self, n):
        raise TypeError("hard-coded players draw from python's `random` (oracle.hardcoded.PyRandomRNG)")

    def choice_uniform(self):
        # np.random.choice(a, p=p) with size=None draws exactly one random_sample()
        # after validating p (numpy mtrand.pyx RandomState.choice); see _choice below.
        return np.random.random_sample()


class TapeRNG:
    """Replays a flat stream of doubles in consumption order."""

    def __init__(self, stream):
        self.s = np.asarray(stream, dtype=np.float64)
        self.i = 0

    def _take(self, k):
        if self.i + k > len(self.s):
            raise IndexError("RNG tape exhausted")
        out = self.s[self.i:self.i + k]
        self.i += k
        return out

    def dirichlet(self, alpha, k):
        return self._take(k).copy()

    def rand(self, k):
        return self._take(k).copy()

    def choice_uniform(self):
        return float(self._take(1)[0])

    def choice_index(self, n):  # hard-coded players: floor(u * n) (the arena's form)
        return min(n - 1, int(float(self._take(1)[0]) * n))


class RecordingRNG:
    """Wraps another RNG and records every double it hands out (the HIP tape format)."""

    def __init__(self, inner):
        self.inner = inner
        self.tape = []

    def dirichlet(self, alpha, k):
        v = self.inner.dirichlet(alpha, k)
        self.tape.extend(float(x) for x in v)
        return v

    def rand(self, k):
        v = self.inner.rand(k)
        self.tape.extend(float(x) for x in v)
        return v

    def choice_uniform(self):
        u = self.inner.choice_uniform()
        self.tape.append(float(u))
        return u

    def choice_index(self, n):
        k = self.inner.choice_index(n)
        self.tape.append((k + 0.5) / n)
        return k


def _kahan_sum(p):
    """numpy's kahan_sum used by RandomState.choice to validate p."""
    if len(p) == 0:
        return 0.0
    s = p[0]
    c = 0.0
    for i in range(1, len(p)):
        y = p[i] - c
        t = s + y
        c = (t - s) - y
        s = t
    return s


def _choice(rng, n, p):
    """np.random.choice(n, p=p) (legacy RandomState) restated: validate, cdf, searchsorted right.

    Returns None where numpy raises ValueError (mcts.py:290-295 then falls back to argmax n).
    """
    p = np.asarray(p, dtype=np.float64)
    atol = math.sqrt(np.finfo(np.float64).eps)
    if np.logical_or.reduce(p < 0):
        return None
    if abs(_kahan_sum(p) - 1.0) > atol:
        return None
    cdf = p.cumsum()
    cdf /= cdf[-1]
    u = rng.choice_uniform()
    return int(cdf.searchsorted(u, side="right"))


def _as_torch_scalar(q):
    """dtype of `torch.tensor(root.q)` (mcts.py:287): a Python float becomes float32, but a
    numpy float64 (root.w turns np.float64 once a strong_play terminal value, computed from
    np.sum at mcts.py:308-311, was added into it) stays float64."""
    if isinstance(q, np.floating):
        return np.float64(q)
    return np.float32(q)


# --------------------------------------------------------------------------- nodes
class Node:
    """MCNode fields (mcts.py:24-47) minus the threading lock (sequential mode)."""

    __slots__ = ("n", "w", "p", "x", "cpuct", "player", "valid", "vl", "noise_active", "p_noise",
                 "children", "state", "v", "locked")

    def __init__(self, p=0.0, player=1, valid=True, x=0.25, cpuct=4):
        self.n = 0
        self.w = 0
        self.p = p
        self.x = x
        self.cpuct = cpuct
        self.player = player
        self.valid = valid
        self.vl = 0
        self.noise_active = False
        self.p_noise = 0
        self.children = ()
        self.state = None
        self.v = None
        self.locked = False  # threading.Lock held while a threaded search waits for the network

    def q(self):  # mcts.py:59-62
        n_eff = self.n + self.vl
        return (self.w - self.vl) / n_eff if n_eff else 0

    def p_eff(self):  # mcts.py:64-69
        if self.noise_active:
            return self.p_noise * self.x + self.p * (1 - self.x)
        return self.p

    def u(self, parent):  # mcts.py:71-78
        return self.cpuct * self.p_eff() * np.sqrt(parent.n + parent.vl) / (1 + self.n + self.vl)

    def select_prob(self, parent):  # mcts.py:80-84
        return -1 * self.player * self.q() + self.u(parent)

    def create_children(self, probs, validities):  # mcts.py:103-107 (order = action index)
        self.children = tuple(
            Node(p=probs[i], player=-self.player, valid=bool(validities[i]), x=self.x, cpuct=self.cpuct)
            for i in range(len(probs))
        )

    def is_leaf(self):
        return len(self.children) == 0


# ---------------------------------------------------------------------------- tree
class OracleTree:
    """MCTreeSearch (mcts.py:116-394), sequential mode, inference only."""

    def __init__(self, game, network, rng, iterations=100, alpha=1, strong_play=False, cpuct=4, x=0.25,
                 evaluate=False, root_player=1, threads=1):
        self.game = game
        self.env_proto = make_env(game)
        self.A = self.env_proto.n_actions
        self.network = network
        self.rng = rng
        self.iterations = iterations
        self.alpha = alpha
        self.strong_play = strong_play
        self.cpuct = cpuct
        self.x = x
        self.evaluating = evaluate
        self.threads = max(1, int(threads))
        self.temp_memory = []
        self.stats = dict(sims=0, nn_evals=0, terminal_leaves=0, depth_sum=0, set_node_expansions=0, leaks=0)
        self.reset(root_player)

    def reset(self, player=1):  # mcts.py:166-174
        env = make_env(self.game)
        base_state = env.reset()
        probs, v = self.network(base_state)  # player defaults to 1 (mcts.py:168)
        self.stats["nn_evals"] += 1
        root = Node(player=player, x=self.x, cpuct=self.cpuct)
        root.state = base_state
        root.v = v
        root.create_children(probs, env.valid_moves())
        self.root = root
        self.moves_played = 0
        self.temp_memory = []
        return base_state

    # -- one move ------------------------------------------------------------
    def move(self):  # __call__ / _search_and_play (mcts.py:177-186)
        self.search()
        return self._play(1)

    def search(self):  # mcts.py:323-338
        self._add_noise(self.root)
        if self.threads > 1:  # mcts.py:328-331: thread_count threads over `iterations` tasks
            slots = [None] * self.threads
            started = 0

            def fill(j):
                nonlocal started
                while started < self.iterations:
                    started += 1
                    item = self._select_threaded()
                    if item is not None:
                        slots[j] = item
                        return

            for j in range(self.threads):
                fill(j)
            while any(x is not None for x in slots):
                # the network answers every pending leaf; the replies are completed oldest-first
                for j in range(self.threads):
                    if slots[j] is not None:
                        item, slots[j] = slots[j], None
                        self._reply_threaded(*item)
                    fill(j)
        else:
            for _ in range(self.iterations):
                self.search_node()
        for c in self.root.children:
            c.noise_active = False

    def _select_threaded(self):
        """search_node (mcts.py:340-367) up to the network call; returns the pending leaf or None."""
        node = self.root
        path = []
        depth = 0
        while True:
            path.append(node)
            node.vl += 1
            scores = [c.select_prob(node) if c.valid and not c.locked else -10000000000 for c in node.children]
            if all(s < -100000 for s in scores):
                self.stats["leaks"] += 1
                return None  # mcts.py:349-354 (the virtual loss stays)
            action = int(np.argmax(scores + 0.000001 * self.rng.rand(self.A)))
            child = node.children[action]
            if child.is_leaf():
                self.stats["sims"] += 1
                self.stats["depth_sum"] += depth + 1
                env = make_env(self.game)
                env.set_state(node.state.copy())
                s, r, done, _ = env.step(action, player=node.player)
                r = r * node.player
                if done:  # _expand_node's terminal branch: no network call, backup at once
                    if self.strong_play:
                        num_steps = np.sum(np.abs(node.state)) + 1
                        v = (1.18 - (9 * num_steps / 350)) * r
                    else:
                        v = r
                    self.stats["terminal_leaves"] += 1
                    child.state = s
                    self._backup_threaded(child, path, v)
                    return None
                child.locked = True  # mcts.py:359
                return child, path, s, env.valid_moves(), node.player
            node = child
            depth += 1

    def _reply_threaded(self, child, path, s, valid, parent_player):
        probs, v = self.network(s, parent_player)  # mcts.py:316
        self.stats["nn_evals"] += 1
        child.create_children(probs, valid)
        child.state = s
        self._backup_threaded(child, path, v)
        child.locked = False

    @staticmethod
    def _backup_threaded(leaf, path, v):  # mcts.py:361-365
        leaf.n += 1
        leaf.w += v
        for a in path:
            a.n += 1
            a.w += v
        leaf.v = v
        for a in path:
            a.vl -= 1
            assert a.vl >= 0

    def _add_noise(self, node):  # mcts.py:49-53
        d = self.rng.dirichlet(self.alpha, len(node.children))
        for i, c in enumerate(node.children):
            c.noise_active = True
            c.p_noise = d[i]

    def search_node(self):  # mcts.py:340-367
        node = self.root
        path = []
        depth = 0
        while True:
            path.append(node)
            node.vl += 1
            scores = [c.select_prob(node) if c.valid else -10000000000 for c in node.children]
            if all(s < -100000 for s in scores):
                return  # (leaks the virtual loss exactly like the reference)
            action = int(np.argmax(scores + 0.000001 * self.rng.rand(self.A)))
            child = node.children[action]
            if child.is_leaf():
                leaf, v = self._expand(node, action, node.player)
                leaf.n += 1
                leaf.w += v
                for a in path:  # backup (mcts.py:94-98), path = ancestors up to the active root
                    a.n += 1
                    a.w += v
                leaf.v = v
                for a in path:
                    a.vl -= 1
                    assert a.vl >= 0
                self.stats["sims"] += 1
                self.stats["depth_sum"] += depth + 1
                break
            node = child
            depth += 1

    def _expand(self, parent, action, player):  # mcts.py:301-321
        env = make_env(self.game)
        env.set_state(parent.state.copy())
        s, r, done, _ = env.step(action, player=player)
        r = r * player
        child = parent.children[action]
        if done:
            if self.strong_play:
                num_steps = np.sum(np.abs(parent.state)) + 1
                v = (1.18 - (9 * num_steps / 350)) * r
            else:
                v = r
            self.stats["terminal_leaves"] += 1
        else:
            probs, v = self.network(s, parent.player)
            self.stats["nn_evals"] += 1
            child.create_children(probs, env.valid_moves())
        child.state = s
        return child, v

    def _play(self, temp=0.05):  # mcts.py:272-299
        if self.evaluating:
            temp = temp / 20
        play_probs = [np.power(c.n, 1 / temp) for c in self.root.children]
        play_probs = play_probs / sum(play_probs)
        action = _choice(self.rng, self.A, play_probs)
        record = None
        if action is None:
            ns = [c.n for c in self.root.children]
            action = ns.index(max(ns))
        else:
            record = dict(
                state=self.root.state.copy(),
                tree_probs=np.asarray(play_probs, dtype=np.float64).astype(np.float32),
                q=_as_torch_scalar(self.root.q()),
            )
            self.temp_memory.append(record)
        self.moves_played += 1
        return action

    # -- tree reuse ------------------------------------------------------------
    def play_action(self, action):  # mcts.py:188-209 (_set_node)
        node = self.root.children[action]
        if node.n == 0:
            node, v = self._expand(self.root, action, self.root.player)
            node.n += 1  # backup (ancestors above the new root are dead)
            node.w += v
            node.v = v
            self.stats["set_node_expansions"] += 1
        self.root = node

    def push_result(self, r):  # push_to_queue (mcts.py:225-232)
        out = [dict(m, actual_val=np.float32(r)) for m in self.temp_memory]
        self.temp_memory = []
        return out

    def root_stats(self):
        kids = self.root.children
        return dict(child_n=[c.n for c in kids], child_w=[float(c.w) for c in kids],
                    root_n=self.root.n, root_w=float(self.root.w))
