"""Device ops on torch tensors, backed by the hand-written gfx950 kernels in
``brpc_amd/csrc/gpu/kernels.hip``. No fallback path: a CPU tensor or a
missing extension raises."""
from .crc32c import crc32c, crc32c_batch, crc32c_host, crc32c_packed  # noqa: F401
from .varint import varint_decode, varint_encode, varint_encode_host, varint_decode_host  # noqa: F401
from .copy import batched_copy, batched_copy_crc32c  # noqa: F401
from .pb import pb_scan  # noqa: F401
from .snappy import snappy_compress, snappy_compress_blocks, snappy_decompress, snappy_decompress_streams  # noqa: F401,E501
from .json import json_index, json_index_host  # noqa: F401
