"""Build, flag and metric helpers."""
from .build import build_native, native_built  # noqa: F401
from .flags import set_flag, get_flag, list_flags  # noqa: F401
from .metrics import dump_vars, dump_prometheus  # noqa: F401
