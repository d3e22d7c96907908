"""Echo workloads used by bench.py and the tests.

ECHO_32B mirrors the reference's headline point (docs/cn/benchmark.md:92-98:
50 synchronous client threads, one connection, 32-byte body);
ECHO_64KB is the large-body point BASELINE.json asks for (the reference's
nearest published one is 32 KB).
"""
from dataclasses import dataclass, asdict

from ..native import native


@dataclass
class EchoWorkload:
    name: str
    request_size: int          # bytes of EchoRequest.message
    attachment_size: int       # bytes of attachment
    concurrency: int = 50      # closed-loop in-flight calls per client
    requests_per_step: int = 20000
    connection_type: str = "single"
    device_attachment: bool = False

    def press_options(self, server, gpu_device=-1, check=False):
        return {
            "server": server,
            "concurrency": self.concurrency,
            "request_size": self.request_size,
            "attachment_size": self.attachment_size,
            "connection_type": self.connection_type,
            "device_attachment": self.device_attachment,
            "gpu_device": gpu_device,
            "check_echo": check,
            "timeout_ms": 5000,
            "max_retry": 0,
        }

    def payload_bytes(self):
        return self.request_size + self.attachment_size

    def asdict(self):
        return asdict(self)


# 32 B message, no attachment
ECHO_32B = EchoWorkload("echo_32B", request_size=32, attachment_size=0, requests_per_step=150000)
# 64 KiB body: tiny message + 64 KiB attachment (zero-copy Buf path)
ECHO_64KB = EchoWorkload("echo_64KB", request_size=16, attachment_size=65536 - 16, requests_per_step=20000)


def start_echo_server(addr="127.0.0.1:0", num_threads=-1, gpu_device=-1, max_concurrency=0):
    s = native.Server()
    s.add_echo_service()
    s.start(addr, num_threads=num_threads, gpu_device=gpu_device, max_concurrency=max_concurrency)
    return s
