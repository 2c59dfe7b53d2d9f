"""Minimal `colorama` stand-in (render-only dependency of the reference envs)."""


def init(*args, **kwargs):
    pass


class Fore:
    GREEN = ""
    RED = ""
    BLUE = ""


class Style:
    RESET_ALL = ""
