"""p2pdl_amd -- MI355X-native drop-in for P2PDL's aggregation / digest hot path.

Layout (only what the path needs):
  csrc/            hand-written HIP kernels for gfx950 + the C ABI (include/p2pdl.h)
  _native.py       ctypes binding; fails loudly when the library / GPU is missing
  ops.py           tensor-level wrappers (FedAvg, median, trimmed mean, SHA-256)
  aggregator/      drop-in for reference aggregator/aggregation.py
  utils/           drop-ins for reference utils/waiting.py and the digest part of utils/crypto.py
  sharded.py       coordinate sharding across GPUs + RCCL all-gather
"""
__all__ = ["ops", "aggregator", "utils", "sharded"]
__version__ = "0.1.0"
