"""`MCTreeSearch` with the reference policy protocol, backed by the HIP arena.

Drop-in for games/algos/mcts.py:116-394.  Same constructor (plus the stale
`env_gen=` / `evaluator=` aliases its own callers still pass,
run_self_play_connect4.py:29, c4_manual.py:24-31), same methods:
`__call__`, `reset`, `play_action`, `push_to_queue`, `pull_from_queue`,
`update_from_memory`, `loss`, `state_dict`, `load_state_dict`, `train`,
`evaluate`, `deduplicate`, attributes `memory`, `memory_queue`, `root_node`,
`env`, `network`, `strong_play`, `temp_memory`.

A single MCTreeSearch drives a one-tree arena (the object tree of mcts.py
becomes the device node store; `root_node` is a read-only view of it).  The
batched self-play path does not go through this class: SelfPlayScheduler
runs thousands of trees per arena (engine.py).
"""
import logging
import time
from collections import namedtuple

import numpy as np
import torch

from .arena import GAMES, Arena, game_of_env
from .base_model import Policy
from .evaluator import make_evaluator

Move = namedtuple("Move", ("state", "actual_val", "tree_probs", "q"))


class _ChildView:
    def __init__(self, n, w, p, player):
        self.n, self.w, self.p, self.player = n, w, p, player

    @property
    def q(self):
        return self.w / self.n if self.n else 0


class RootView:
    """Read-only snapshot of the active root (MCNode fields n, w, q, player, state, children)."""

    def __init__(self, stats):
        self.n = stats["root_n"]
        self.w = stats["root_w"]
        self.player = stats["root_player"]
        self.state = stats["board"].astype(np.int64)
        self.children = tuple(_ChildView(n, w, p, -self.player)
                              for n, w, p in zip(stats["child_n"], stats["child_w"], stats["child_p"]))

    @property
    def q(self):
        return self.w / self.n if self.n else 0


def az_loss(network, states, actual_val, tree_probs, q, q_average=True):
    """The AlphaZero loss of MCTreeSearch.loss (mcts.py:234-252) on stacked tensors:
    MSELossFlat(v, z [+ q]) (rl_utils/flat.py: float targets, mean over the batch) plus
    -sum(pi * log p) / B.  `states` int64 [B, W, H] in the Move frame (+1 = player to move).
    Shared by MCTreeSearch.loss and the scheduler's trainer (self_play_parallel._Trainer);
    pinned by tests/golden/trainer_step.npz (G8)."""
    dev = next(network.parameters()).device
    probs, value = network.forward(states.to(dev))
    z = actual_val.to(dev).float()
    if q_average:
        z = z + q.to(dev)
    value_loss = torch.mean((value.reshape(-1) - z.float().reshape(-1)) ** 2)
    prob_loss = -(probs.log() * tree_probs.to(dev)).sum() / probs.size()[0]
    return value_loss + prob_loss


class MCTreeSearch(Policy):
    def __init__(self, network=None, env=None, optim=None, memory_queue=None, iterations=100, temperature_cutoff=5,
                 batch_size=64, memory_size=200000, min_memory=20000, update_nn=True, starting_state_dict=None,
                 thread_count=4, strong_play=False, q_average=True, alpha=1, env_gen=None, evaluator=None,
                 seed=None, device=None, rng="philox", cpuct=4, x_noise=0.25, threading=False):
        network = network if network is not None else evaluator
        env = env if env is not None else env_gen
        if network is None or env is None:
            raise TypeError("MCTreeSearch needs `network` and `env` (or the legacy `evaluator` / `env_gen`)")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        if isinstance(network, torch.nn.Module):
            network = network.to(self.device)
        self.network = network
        self.env_gen = env
        self.env = env() if callable(env) else env
        self.game = game_of_env(self.env)
        _, self.W, self.H, self.actions = GAMES[self.game]
        self.optim = optim
        self.iterations = iterations
        self.alpha = alpha
        self.strong_play = strong_play
        self.q_average = q_average
        self.batch_size = batch_size
        self.min_memory = min_memory
        self.temperature_cutoff = temperature_cutoff
        self.update_nn = update_nn
        self.starting_state_dict = starting_state_dict
        self.thread_count = thread_count
        self.evaluating = False
        # threading=True: thread_count sims in flight with virtual loss, the reference's mode when its
        # network is an InferenceProxy (mcts.py:154, :328-331); False: its sequential mode
        self.threading = bool(threading)
        k = int(thread_count) if self.threading and thread_count and thread_count > 1 else 1
        # fp16 trunk: the reference's inference autocast dtype (inference_worker.py:114-119)
        self._evaluator = make_evaluator(network, self.game, device=self.device, dtype=torch.float16)
        if seed is None:
            seed = int(np.random.randint(0, 2**31 - 1))
        self._arena = Arena(self.game, n_trees=1, n_games=0, iterations=iterations, rng=rng, seed=seed,
                            strong_play=strong_play, leaf_format=self._evaluator.leaf_format,
                            leaf_layout=self._evaluator.leaf_layout, cpuct=cpuct, x_noise=x_noise, alpha=alpha,
                            device=self.device, search_threads=k)
        self.temp_memory = []
        self.moves_played = 0
        # weights changed (update_from_memory / load_state_dict): the evaluator's folded / packed copy is
        # refreshed before the next leaf evaluation, the empty-board root prior at the next reset
        self._weights_stale = False
        self._root_prior_stale = True
        if starting_state_dict:
            self.load_state_dict(starting_state_dict)
        super().__init__(memory_queue=memory_queue, memory_size=memory_size)
        self.reset()

    # ------------------------------------------------------------------ search
    def _sync_weights(self):
        """The reference evaluates every leaf with the network as it is now (mcts.py:316): after an
        update the evaluator's packed weights are re-derived before the next evaluation."""
        if self._weights_stale:
            if hasattr(self._evaluator, "refresh"):
                self._evaluator.refresh()
            self._weights_stale = False

    def _refresh_root_prior(self):
        self._sync_weights()
        x = self._evaluator.empty_root_input(self.W, self.H, self.device)
        probs, _ = self._evaluator(x)
        self._arena.set_root_prior(probs[0])
        self._root_prior_stale = False

    def _eval_expand(self, n):
        if n:
            self._sync_weights()
            probs, values = self._evaluator(self._arena.leaves(n))
            self._arena.expand(probs, values)

    def reset(self, player=1):
        """mcts.py:166-174"""
        if self._root_prior_stale:
            self._refresh_root_prior()
        self._arena.tree_reset([0], [player])
        self.moves_played = 0
        self.temp_memory = []
        self._arena.check()
        return np.zeros([self.W, self.H], dtype=np.int64)

    def __call__(self, s=None):
        """Search `iterations` simulations from the root and pick a move (mcts.py:177-186)."""
        self.search()
        return self._play(1)

    def search(self):
        a = self._arena
        a.search_begin([0])
        for _ in range(-(-self.iterations // a.search_threads)):
            self._eval_expand(a.select())

    def _play(self, temp=1):
        if self.evaluating:
            temp = temp / 20  # mcts.py:273-274
        out = self._arena.search_end(temp)
        action = int(out["action"][0])
        if int(out["recorded"][0]):
            q = float(out["q"][0])
            qt = torch.tensor(q, dtype=torch.float64) if int(out["q_f64"][0]) else torch.tensor(q, dtype=torch.float32)
            self.temp_memory.append(Move(
                torch.as_tensor(out["state"][0].cpu().numpy().astype(np.int64).reshape(self.W, self.H)),
                None, out["tree_probs"][0].cpu().clone(), qt))
        else:
            logging.info("action exception: falling back to the most visited child")
        self.moves_played += 1
        self._arena.check()
        return action

    def play_action(self, action, player=None):
        """Advance the root; an unvisited child is expanded and backed up (mcts.py:188-209)."""
        self._eval_expand(self._arena.play_action([0], [int(action)]))

    @property
    def root_node(self):
        return RootView(self._arena.root_stats(0))

    # ------------------------------------------------------------------ memory / training
    def update(self, s, a, r, done, next_s):
        self.push_to_queue(s, a, r, done, next_s)
        self.pull_from_queue()
        if self.ready:
            self.update_from_memory()

    def pull_from_queue(self):
        while not self.memory_queue.empty():
            e = self.memory_queue.get()
            self.memory.add(Move(*[e[i].to(self.device) for i in range(4)]))

    def push_to_queue(self, s=None, a=None, r=None, done=None, next_s=None):
        """mcts.py:225-232: on `done`, stamp the owner's result on every buffered Move."""
        if done:
            for e in self.temp_memory:
                self.memory_queue.put(e._replace(actual_val=torch.tensor(r).float()))
            self.temp_memory = []

    def loss(self, batch):
        """AlphaZero loss (mcts.py:234-252): MSE(v, z [+ q]) - sum(pi * log p) / B."""
        s, actual_val, tree_probs, q = Move(*zip(*batch))
        return az_loss(self.network, torch.stack(s), torch.stack(actual_val), torch.stack(tree_probs),
                       torch.stack(q), self.q_average)

    def update_from_memory(self):
        if len(self.memory) < self.batch_size:
            time.sleep(1)
            return
        loss = self.loss(self.memory.sample(self.batch_size))
        self.optim.zero_grad()
        loss.backward()
        self.optim.step()
        self._weights_stale = True
        self._root_prior_stale = True

    @property
    def ready(self):
        return len(self.memory) >= self.min_memory and self.update_nn

    def load_state_dict(self, state_dict, target=False):
        self.network.load_state_dict(state_dict)
        self._weights_stale = True
        self._root_prior_stale = True

    def state_dict(self):
        return self.network.state_dict()

    def update_target_net(self):
        pass

    def deduplicate(self):
        self.memory.deduplicate("state", ["actual_val", "tree_probs"], Move)

    def train(self, train_state=True):
        if hasattr(self.network, "train"):
            return self.network.train(train_state)
        return self.network

    def evaluate(self, evaluate_state=False):
        """Evaluate mode plays with temp / 20 (mcts.py:273-274, :392-394)."""
        self.evaluating = evaluate_state
