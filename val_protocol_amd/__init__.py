"""val_protocol_amd -- MI355X-native CRC-32 integrity path of the VAL protocol.

The product is ``libval_crc_hip.so`` (HIP kernels for gfx950 + a C ABI,
``include/val_crc32_gpu.h``). ``crc`` and ``wire`` are ctypes bindings used by
tests and bench.py; they never compute a CRC on the CPU.
"""
from . import crc, wire  # noqa: F401
from .crc import (  # noqa: F401
    LIB_PATH, ValError, crc32_combine, crc32_provider, crc32_shift, frames, frames_host, region,
    val_crc32, val_crc32_finalize_state, val_crc32_init_state, val_crc32_update_state, verify_frames,
    verify_frames_host,
)

__version__ = "0.1.0"
