"""Workload definitions ("model families" of an RPC framework): the echo
service configurations the reference benchmarks (example/echo_c++,
multi_threaded_echo_c++, streaming_echo_c++) as reusable specs."""
from .echo import EchoWorkload, ECHO_32B, ECHO_64KB, start_echo_server  # noqa: F401
