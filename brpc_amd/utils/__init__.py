"""Build, flag and metric helpers."""
from .build import build_native, native_built  # noqa: F401
from .flags import (set_flag, get_flag, get_flag_typed, list_flags, parse_flag_args, apply_flag_args,  # noqa: F401
                    apply_env_flags, flag_overrides)
from .metrics import dump_vars, dump_prometheus, parse_prometheus, VarSnapshot, wait_for_var  # noqa: F401
