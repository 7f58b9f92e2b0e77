"""coala_amd — MI355X (gfx950) model-update codec for COALA's federated sync path.

Hot path: CodecSpec v1 encode/decode as hand-written HIP kernels (coala_amd/csrc/coalac.hip) behind a
C ABI (include/coalac.h), reached from Python via ctypes (coala_amd/compression/_lib.py).
"""
__version__ = "0.1.0"
