"""Exposed metrics (the bvar analog)."""
from ..native import native


def dump_vars(filter=""):
    """name -> value text for every exposed variable matching ``filter``
    (wildcards ``*``/``?``, ``;``-separated alternatives)."""
    return native.dump_vars(filter)


def dump_prometheus():
    return native.dump_prometheus()
