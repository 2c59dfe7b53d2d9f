"""Policy plug-in protocol and the policy factory, as the scheduler sees them.

Same names and call signatures as games/general/base_model.py:10-100, so a
reference `ModelContainer(policy_gen=MCTreeSearch, ...)` drives this package's
`MCTreeSearch` and the hard-coded players unchanged.  The methods a concrete
player must provide raise NotImplementedError (as in the reference); the
optional hooks are no-ops.
"""
import torch

from .memory import Memory


def _abstract(name):
    def method(self, *args, **kwargs):
        raise NotImplementedError(f"{type(self).__name__}.{name}")

    method.__name__ = name
    return method


class BasePlayer:
    """Anything that can play a game (base_model.py:10-25).

    __call__(s) -> action, reset(player=1), play_action(action, player) are required;
    train(flag) and evaluate(flag=False) are optional hooks."""

    __call__ = _abstract("__call__")
    reset = _abstract("reset")
    play_action = _abstract("play_action")

    def train(self, train_state):
        return None

    def evaluate(self, evaluate_state=False):
        return None


class TrainableModel:
    """A player with a replay memory fed from a queue (base_model.py:28-72)."""

    def __init__(self, memory_queue=None, memory_size=None, *args, **kwargs):
        self.memory_queue = memory_queue
        self.memory = self.create_memory(memory_size)

    def create_memory(self, memory_size):
        return Memory(memory_size)

    load_state_dict = _abstract("load_state_dict")
    update_from_memory = _abstract("update_from_memory")
    state_dict = _abstract("state_dict")
    train = _abstract("train")
    push_to_queue = _abstract("push_to_queue")

    @property
    def ready(self):
        raise NotImplementedError(f"{type(self).__name__}.ready")

    def evaluate(self, evaluate_state=False):
        return None

    def deduplicate(self):
        return None

    def pull_from_queue(self):
        """Drain the memory queue into the replay memory."""
        q = self.memory_queue
        while not q.empty():
            self.memory.add(q.get())

    def update(self, s, a, r, done, next_s):
        """One push / pull / (conditional) learning step."""
        self.push_to_queue(s, a, r, done, next_s)
        self.pull_from_queue()
        if self.ready:
            self.update_from_memory()


class Policy(TrainableModel, BasePlayer):
    pass


class ModelContainer:
    """Deferred policy construction: setup(**kw) == policy_gen(*policy_args, **policy_kwargs, **kw)
    (base_model.py:79-100); the legacy "evaluator" kwarg is renamed to "network"."""

    def __init__(self, policy_gen, policy_args=None, policy_kwargs=None):
        self.policy_gen = policy_gen
        self.policy_args = list(policy_args) if policy_args else []
        self.policy_kwargs = dict(policy_kwargs) if policy_kwargs else {}

    def setup(self, **kwargs):
        kw = self.policy_kwargs
        if "evaluator" in kw:
            kw["network"] = kw.pop("evaluator")
        return self.policy_gen(*self.policy_args, **kw, **kwargs)

    def load_state_dict(self, save_file):
        """Checkpoints are {"model": state_dict}; loaded with weights_only=True."""
        ck = torch.load(save_file, weights_only=True, map_location="cpu")
        self.policy_kwargs["network"].load_state_dict(ck["model"])

    def set_env(self, env):
        self.policy_kwargs["env"] = env
        return self

    def set_network(self, network):
        self.policy_kwargs["network"] = network
        return self
