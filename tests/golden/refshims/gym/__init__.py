"""Minimal `gym` stand-in: only `gym.spaces.Discrete(n).n` is used by the reference envs."""
from . import spaces  # noqa: F401
