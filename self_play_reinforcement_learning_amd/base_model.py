"""Policy plug-in protocol and factory (games/general/base_model.py:10-100)."""
import torch

from .memory import Memory


class BasePlayer:
    def __call__(self, s):
        raise NotImplementedError

    def reset(self, player=1):
        raise NotImplementedError

    def play_action(self, action, player):
        raise NotImplementedError

    def train(self, train_state):
        pass

    def evaluate(self, evaluate_state=False):
        pass


class TrainableModel:
    def __init__(self, memory_queue=None, memory_size=None, *args, **kwargs):
        self.memory = self.create_memory(memory_size)
        self.memory_queue = memory_queue

    def create_memory(self, memory_size):
        return Memory(memory_size)

    def load_state_dict(self, state_dict, target=False):
        raise NotImplementedError

    def update(self, s, a, r, done, next_s):
        self.push_to_queue(s, a, r, done, next_s)
        self.pull_from_queue()
        if self.ready:
            self.update_from_memory()

    def update_from_memory(self):
        raise NotImplementedError

    @property
    def ready(self):
        raise NotImplementedError

    def state_dict(self):
        raise NotImplementedError

    def train(self, train_state):
        raise NotImplementedError

    def evaluate(self, evaluate_state=False):
        pass

    def pull_from_queue(self):
        while not self.memory_queue.empty():
            self.memory.add(self.memory_queue.get())

    def push_to_queue(self, s, a, r, done, next_s):
        raise NotImplementedError

    def deduplicate(self):
        pass


class Policy(TrainableModel, BasePlayer):
    pass


class ModelContainer:
    """ModelContainer(policy_gen, policy_args, policy_kwargs).setup(**kw) (base_model.py:79-100)."""

    def __init__(self, policy_gen, policy_args=None, policy_kwargs=None):
        self.policy_gen = policy_gen
        self.policy_args = list(policy_args or [])
        self.policy_kwargs = dict(policy_kwargs or {})

    def setup(self, **kwargs):
        if "evaluator" in self.policy_kwargs:  # legacy key (base_model.py:86-87)
            self.policy_kwargs["network"] = self.policy_kwargs.pop("evaluator")
        return self.policy_gen(*self.policy_args, **self.policy_kwargs, **kwargs)

    def load_state_dict(self, save_file):
        checkpoint = torch.load(save_file, weights_only=True, map_location="cpu")
        self.policy_kwargs["network"].load_state_dict(checkpoint["model"])

    def set_env(self, env):
        self.policy_kwargs["env"] = env
        return self

    def set_network(self, network):
        self.policy_kwargs["network"] = network
        return self
