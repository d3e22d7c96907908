"""Exposed metrics (the bvar analog, reference src/bvar and the /vars and
/brpc_metrics pages): dumps of every exposed variable, a parser for the
Prometheus text the native side renders, and snapshots that turn counters
into deltas and rates between two points in time."""
import re
import time

from ..native import native

_SAMPLE = re.compile(r'^([a-zA-Z_:][a-zA-Z0-9_:]*)(\{(.*)\})?\s+(\S+)')
_LABEL = re.compile(r'([a-zA-Z_][a-zA-Z0-9_]*)="((?:[^"\\]|\\.)*)"')


def dump_vars(filter=""):
    """name -> value text for every exposed variable matching ``filter``
    (wildcards ``*``/``?``, ``;``-separated alternatives)."""
    return native.dump_vars(filter)


def dump_prometheus():
    """Every variable in the Prometheus text exposition format."""
    return native.dump_prometheus()


def parse_prometheus(text):
    """Prometheus text -> ``{(name, ((label, value), ...)): float}``.
    Comment lines are skipped; label values are unescaped."""
    out = {}
    for line in text.splitlines():
        line = line.strip()
        if not line or line.startswith("#"):
            continue
        m = _SAMPLE.match(line)
        if not m:
            raise ValueError("bad prometheus sample: %r" % line)
        labels = tuple((k, bytes(v, "utf-8").decode("unicode_escape")) for k, v in _LABEL.findall(m.group(3) or ""))
        out[(m.group(1), labels)] = float(m.group(4))
    return out


def _number(text):
    try:
        return float(text)
    except (TypeError, ValueError):
        return None


class VarSnapshot:
    """Numeric variables at one instant (non-numeric ones are dropped)."""

    def __init__(self, filter=""):
        self.t = time.monotonic()
        self.values = {}
        for k, v in dump_vars(filter).items():
            x = _number(v)
            if x is not None:
                self.values[k] = x

    def delta(self, earlier):
        """name -> self - earlier for variables present in both."""
        return {k: v - earlier.values[k] for k, v in self.values.items() if k in earlier.values}

    def rates(self, earlier):
        """name -> per-second change since ``earlier``."""
        dt = self.t - earlier.t
        if dt <= 0:
            raise ValueError("snapshots are not ordered in time")
        return {k: d / dt for k, d in self.delta(earlier).items()}


def wait_for_var(name, predicate, timeout=5.0, interval=0.01):
    """Poll variable ``name`` until ``predicate(value_text)`` holds; returns
    the last value text (raises TimeoutError when it never did)."""
    deadline = time.monotonic() + timeout
    last = None
    while True:
        last = dump_vars(name).get(name)
        if last is not None and predicate(last):
            return last
        if time.monotonic() >= deadline:
            raise TimeoutError("%s never satisfied the predicate (last %r)" % (name, last))
        time.sleep(interval)
