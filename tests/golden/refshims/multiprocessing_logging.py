"""No-op stand-in for `multiprocessing_logging` (logging plumbing only)."""


def install_mp_handler(logger=None):
    pass
