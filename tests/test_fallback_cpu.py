"""Failure policy of the scalar hooks (crc32_func_t has no error
channel, reference include/val_protocol.h:163-166, and VAL calls it under the
session mutex, src/val_core.c:721-836). Run where no GPU exists: the C hooks
answer with the library's own CPU slice-by-8 and count it; the Python API
raises instead (no silent fallback); batch calls return VAL_ERR_IO. Each case
runs in a fresh process so the count starts at zero."""
import os
import subprocess
import sys

import pytest

import val_protocol_amd.crc as vc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = r"""
import ctypes, sys
sys.path.insert(0, {root!r})
import val_protocol_amd.crc as vc
from tests import _oracle, _prng
lib = vc.lib()
data = _prng.prng_bytes(77, 100_003)
p = ctypes.c_void_p(data.ctypes.data)
assert lib.val_gpu_crc32_provider(0xFFFFFFFF, p, data.size) == _oracle.crc32(data)
assert lib.val_crc32(p, 4099) == _oracle.crc32(data[:4099])
assert lib.val_crc32_update_state(0x12345678, p, 17) == _oracle.update_state(0x12345678, data[:17])
assert lib.val_crc32(ctypes.c_char_p(b"123456789"), 9) == 0xCBF43926
assert lib.val_gpu_cpu_fallback_count() == 4
try:
    vc.crc32_provider(0xFFFFFFFF, b"abc")
except vc.ValError as e:
    assert e.status == vc.VAL_ERR_IO
else:
    raise AssertionError("Python API must not return a CPU result silently")
crc = (ctypes.c_uint32 * 1)()
st = lib.val_crc32_frames_host(data.ctypes.data, data.size, None, None, 100, 100, 1, crc, None)
assert st == vc.VAL_ERR_IO, st
print("ok")
"""


def _run(env_extra):
    env = dict(os.environ, **env_extra)
    return subprocess.run([sys.executable, "-c", _SCRIPT.format(root=ROOT)], env=env, capture_output=True, text=True,
                          timeout=300)


def test_scalar_hooks_fall_back_to_cpu_and_count():
    if vc.device_count() > 0:
        pytest.skip("a GPU is present: the GPU suite asserts the count stays 0 instead")
    r = _run({})
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stdout + r.stderr


def test_scalar_hooks_abort_when_fallback_disabled():
    if vc.device_count() > 0:
        pytest.skip("a GPU is present")
    r = _run({"VAL_GPU_CPU_FALLBACK": "0"})
    assert r.returncode != 0 and "CPU fallback disabled" in r.stderr
