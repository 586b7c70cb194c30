"""Python host binding of the MI355X CRC-32 integrity path.

Thin ctypes layer over ``val_protocol_amd/libval_crc_hip.so`` (C ABI declared
in ``include/val_crc32_gpu.h``). Names mirror the reference interface:

* ``val_crc32`` / ``val_crc32_init_state`` / ``val_crc32_update_state`` /
  ``val_crc32_finalize_state`` -- reference ``src/val_core.c:150-183``
* ``crc32_provider`` -- a ``crc32_func_t`` (reference
  ``include/val_protocol.h:163-166``); ``provider_address()`` returns the C
  function pointer to install into ``val_config_t.crc32_provider``
* ``frames`` / ``verify_frames`` -- batched trailer CRC / RX verify of DATA
  frames (reference ``src/val_core.c:828-834`` and ``:963-974``)
* ``region`` -- long-window CRC (reference ``src/val_core.c:414-455``)

Region and device calls compute on the GPU; if the shared library is
missing or the GPU path fails, calls raise (no CPU fallback). By design, the
scalar hooks answer inputs below the provider threshold, and the host-memory
batch calls batches below the host-batch threshold, with the library's own
CPU engine (``provider_min_bytes`` / ``host_batch_min_bytes``; 0 forces the
GPU); above them a failed GPU path raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

VAL_OK = 0
VAL_ERR_INVALID_ARG = -1
VAL_ERR_NO_MEMORY = -2
VAL_ERR_IO = -3
VAL_ERR_CRC = -6

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libval_crc_hip.so")

# Exported symbols (kept in sync with include/*.h; tests/test_abi.py checks).
EXPORTS = (
    "val_gpu_init", "val_gpu_shutdown", "val_gpu_device_count", "val_gpu_abi_version",
    "val_gpu_last_error", "val_gpu_lanes_per_frame", "val_gpu_set_lanes_per_frame",
    "val_gpu_set_prefetch",
    "val_gpu_crc32_provider", "val_crc32_combine", "val_crc32_shift",
    "val_crc32", "val_crc32_init_state", "val_crc32_update_state", "val_crc32_finalize_state",
    "val_crc32_frames_dev", "val_crc32_verify_frames_dev", "val_crc32_region_dev",
    "val_crc32_region_scratch_bytes", "val_crc32_frames_host", "val_crc32_verify_frames_host",
    "val_serialize_frame_header", "val_deserialize_frame_header", "val_frame_data_batch",
    "val_frame_put_trailers", "val_frame_scan", "val_gpu_host_alloc", "val_gpu_host_free",
    "val_gpu_set_host_chunk_bytes", "val_gpu_init_devices", "val_gpu_set_device", "val_gpu_current_device",
    "val_gpu_cpu_fallback_count", "val_gpu_set_cpu_fallback", "val_crc32_frames_host_multi",
    "val_crc32_verify_frames_host_multi", "val_crc32_region_host_multi", "val_shard_frames", "val_crc32_fold_partials",
    "val_crc32_verify_frames_ex_dev", "val_crc32_verify_frames_ex_host", "val_crc32_fold_payload_states",
    "val_frame_payload_lens", "val_gpu_set_provider_min_bytes", "val_gpu_provider_min_bytes",
    "val_gpu_cpu_small_count", "val_gpu_last_hook_path", "val_crc32_cpu_update_state", "val_crc32_cpu_engine",
    "val_crc32_fold_payload_states_at", "val_frame_data_offsets", "val_gpu_build_flags",
    "val_gpu_host_copy_threads", "val_gpu_host_copy_probe", "val_gpu_set_ragged_min_frames", "val_gpu_ragged_min_frames",
    "val_gpu_scratch_entries", "val_gpu_set_host_batch_min_bytes", "val_gpu_host_batch_min_bytes",
    "val_gpu_host_batch_min_bytes_for",
    "val_gpu_cpu_batch_count", "val_gpu_set_host_cpu_threads", "val_gpu_host_multi_min_bytes", "val_gpu_host_multi_min_bytes_ex",
    "val_gpu_set_tail_pieces", "val_gpu_tail_piece_launches",
    "val_batch_attach", "val_batch_flush", "val_batch_get_stats", "val_batch_detach", "val_batch_crc32_provider",
    "val_serialize_handshake", "val_deserialize_handshake", "val_serialize_meta", "val_deserialize_meta",
    "val_serialize_resume_resp", "val_deserialize_resume_resp", "val_serialize_verify_request",
    "val_deserialize_verify_request", "val_serialize_verify_response", "val_deserialize_verify_response",
    "val_serialize_error_payload", "val_deserialize_error_payload",
)

# Where the calling thread's last scalar-hook call was answered (val_gpu_last_hook_path).
HOOK_NONE, HOOK_GPU, HOOK_CPU, HOOK_FALLBACK = 0, 1, 2, 3


class ValError(RuntimeError):
    def __init__(self, status: int, where: str, detail: str = ""):
        super().__init__(f"{where} failed: status {status} {detail}".strip())
        self.status = status


_lib: Optional[ctypes.CDLL] = None

_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p


def _declare(lib: ctypes.CDLL, strict: bool = True) -> None:
    """Set argument and result types; strict=False skips symbols an older
    build lacks (A/B tooling loads libraries of earlier revisions)."""
    def fn(name, res, *args):
        if not strict and not hasattr(lib, name):
            return
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = list(args)

    i32, u32, u64, sz = ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_size_t
    fn("val_gpu_init", i32, ctypes.c_int)
    fn("val_gpu_shutdown", None)
    fn("val_gpu_device_count", ctypes.c_int)
    fn("val_gpu_abi_version", u32)
    fn("val_gpu_last_error", ctypes.c_char_p)
    fn("val_gpu_lanes_per_frame", u32, u32)
    fn("val_gpu_set_lanes_per_frame", i32, u32)
    fn("val_gpu_set_prefetch", i32, ctypes.c_int)
    fn("val_gpu_crc32_provider", u32, u32, _vp, sz)
    fn("val_crc32_combine", u32, u32, u32, u64)
    fn("val_crc32_shift", u32, u32, u64)
    fn("val_crc32", u32, _vp, sz)
    fn("val_crc32_init_state", u32)
    fn("val_crc32_update_state", u32, u32, _vp, sz)
    fn("val_crc32_finalize_state", u32, u32)
    fn("val_crc32_frames_dev", i32, _vp, _vp, _vp, u64, u32, u32, u32, _vp, _vp, _vp)
    fn("val_crc32_verify_frames_dev", i32, _vp, _vp, _vp, u64, u32, u32, u32, _vp, _vp, _vp, _vp, _vp)
    fn("val_crc32_region_dev", i32, _vp, u64, u32, _vp, _vp)
    fn("val_crc32_region_scratch_bytes", u64, u64)
    fn("val_crc32_frames_host", i32, _vp, u64, _vp, _vp, u64, u32, u32, _vp, _vp)
    fn("val_crc32_verify_frames_host", i32, _vp, u64, _vp, _vp, u64, u32, u32, _vp, _vp)
    fn("val_serialize_frame_header", None, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint16, u32, _vp)
    fn("val_deserialize_frame_header", None, _vp, _vp, _vp, _vp, _vp)
    fn("val_frame_data_batch", i32, _vp, _vp, _vp, _vp, _vp, u32, _vp, sz, _vp, _vp, ctypes.POINTER(sz))
    fn("val_frame_put_trailers", None, _vp, _vp, _vp, _vp, u32)
    fn("val_frame_scan", i32, _vp, sz, sz, u32, _vp, _vp, ctypes.POINTER(u32), ctypes.POINTER(sz))
    fn("val_gpu_host_alloc", _vp, sz)
    fn("val_gpu_host_free", None, _vp)
    fn("val_gpu_set_host_chunk_bytes", i32, sz)
    fn("val_gpu_init_devices", ctypes.c_int, ctypes.c_int)
    fn("val_gpu_set_device", i32, ctypes.c_int)
    fn("val_gpu_current_device", ctypes.c_int)
    fn("val_gpu_cpu_fallback_count", u64)
    fn("val_gpu_set_cpu_fallback", None, ctypes.c_int)
    fn("val_crc32_frames_host_multi", i32, _vp, u64, _vp, _vp, u64, u32, u32, _vp, _vp, ctypes.c_int)
    fn("val_crc32_verify_frames_host_multi", i32, _vp, u64, _vp, _vp, u64, u32, u32, _vp, _vp, ctypes.c_int)
    fn("val_crc32_region_host_multi", i32, _vp, u64, u32, _vp, ctypes.c_int)
    fn("val_shard_frames", None, u32, _vp, u32, u32, ctypes.POINTER(u32), ctypes.POINTER(u32))
    fn("val_crc32_fold_partials", u32, _vp, _vp, u32)
    fn("val_crc32_verify_frames_ex_dev", i32, _vp, _vp, _vp, u64, u32, u32, u32, _vp, _vp, _vp, _vp, _vp, _vp)
    fn("val_crc32_verify_frames_ex_host", i32, _vp, u64, _vp, _vp, u64, u32, u32, _vp, _vp, _vp)
    fn("val_crc32_fold_payload_states", u32, u32, _vp, _vp, _vp, u32, ctypes.POINTER(u32))
    fn("val_frame_payload_lens", None, _vp, _vp, _vp, u32, _vp)
    fn("val_gpu_set_provider_min_bytes", None, ctypes.c_int64)
    fn("val_gpu_provider_min_bytes", u64)
    fn("val_gpu_cpu_small_count", u64)
    fn("val_gpu_last_hook_path", ctypes.c_int)
    fn("val_crc32_cpu_update_state", u32, u32, _vp, sz, ctypes.c_int)
    fn("val_crc32_cpu_engine", ctypes.c_int)
    fn("val_crc32_fold_payload_states_at", u32, u32, _vp, _vp, _vp, _vp, u32, ctypes.POINTER(u64),
       ctypes.POINTER(u32))
    fn("val_frame_data_offsets", None, _vp, _vp, _vp, u32, _vp)
    fn("val_gpu_build_flags", ctypes.c_char_p)
    fn("val_gpu_host_copy_threads", u32, u64, u32)
    fn("val_gpu_host_copy_probe", i32, u32, u64, u32, ctypes.c_int, ctypes.POINTER(ctypes.c_double))
    fn("val_gpu_set_ragged_min_frames", None, ctypes.c_int64)
    fn("val_gpu_ragged_min_frames", u32)
    fn("val_gpu_scratch_entries", u32, ctypes.c_int, ctypes.POINTER(u64))
    fn("val_gpu_set_host_batch_min_bytes", None, ctypes.c_int64)
    fn("val_gpu_host_batch_min_bytes", u64)
    fn("val_gpu_host_batch_min_bytes_for", u64, u64)
    fn("val_gpu_cpu_batch_count", u64)
    fn("val_gpu_set_host_cpu_threads", None, u32)
    fn("val_gpu_host_multi_min_bytes", u64, ctypes.c_int)
    fn("val_gpu_host_multi_min_bytes_ex", u64, ctypes.c_int, ctypes.c_int, u64)
    fn("val_gpu_set_tail_pieces", None, ctypes.c_int)
    fn("val_gpu_tail_piece_launches", u64)


def lib() -> ctypes.CDLL:
    """Load the HIP shared library. A library that is missing, or was built
    from other sources than this tree's, is (re)built first under a file lock;
    if that fails this raises (there is no CPU fallback)."""
    global _lib
    if _lib is None:
        from . import _build

        try:
            _build.ensure_built()
        except Exception as e:  # noqa: BLE001 - reported with the cause
            raise ImportError(f"{LIB_PATH} could not be built ({e}); no CPU fallback") from e
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: run __graft_entry__.build() first (no CPU fallback)")
        try:  # one HIP runtime per process: let torch's libamdhip64 load first
            import torch  # noqa: F401
        except Exception:  # pragma: no cover - torch is always present in this image
            pass
        l = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
        _declare(l)
        _lib = l
    return _lib


def last_error() -> str:
    return lib().val_gpu_last_error().decode(errors="replace")


def _check(st: int, where: str) -> None:
    if st != VAL_OK:
        raise ValError(st, where, last_error())


def _buf(data) -> tuple[ctypes.c_void_p, int, object]:
    """Host byte buffer -> (pointer, length, keepalive)."""
    if isinstance(data, (bytes, bytearray, memoryview)):
        arr = np.frombuffer(bytes(data) if isinstance(data, memoryview) else data, dtype=np.uint8)
    else:
        arr = np.ascontiguousarray(np.asarray(data).view(np.uint8).reshape(-1))
    return ctypes.c_void_p(arr.ctypes.data if arr.size else 0), int(arr.size), arr


# ---- scalar surface -------------------------------------------------------
def init(device: int = 0) -> None:
    _check(lib().val_gpu_init(device), "val_gpu_init")


def device_count() -> int:
    return int(lib().val_gpu_device_count())


def init_devices(n: int = 0) -> int:
    """Initialise devices 0..n-1 (0: all); returns how many are usable."""
    return int(lib().val_gpu_init_devices(n))


def set_device(device: int) -> None:
    """Bind the calling thread's later calls to `device`."""
    _check(lib().val_gpu_set_device(device), "val_gpu_set_device")


def current_device() -> int:
    return int(lib().val_gpu_current_device())


def cpu_fallback_count() -> int:
    """Scalar-hook calls the C library answered on the CPU after a GPU failure."""
    return int(lib().val_gpu_cpu_fallback_count())


def cpu_small_count() -> int:
    """Scalar-hook calls answered on the CPU because they were below the provider threshold."""
    return int(lib().val_gpu_cpu_small_count())


def last_hook_path() -> int:
    """HOOK_GPU / HOOK_CPU / HOOK_FALLBACK: where this thread's last scalar-hook call ran."""
    return int(lib().val_gpu_last_hook_path())


def set_provider_min_bytes(nbytes: int) -> None:
    """Scalar hooks answer inputs shorter than nbytes on the CPU (0: always the
    GPU; -1: VAL_GPU_PROVIDER_MIN_BYTES or the built-in crossover)."""
    lib().val_gpu_set_provider_min_bytes(int(nbytes))


def provider_min_bytes() -> int:
    return int(lib().val_gpu_provider_min_bytes())


def set_host_batch_min_bytes(nbytes: int) -> None:
    """Host batches with fewer CRC-input bytes than this are answered by the
    CPU engine (0: always the GPU; -1: VAL_GPU_HOST_BATCH_MIN_BYTES or the
    built-in crossover)."""
    lib().val_gpu_set_host_batch_min_bytes(int(nbytes))


def host_batch_min_bytes() -> int:
    return int(lib().val_gpu_host_batch_min_bytes())


def cpu_batch_count() -> int:
    """Host batches answered by the CPU engine because they were below the threshold."""
    return int(lib().val_gpu_cpu_batch_count())


def set_host_cpu_threads(threads: int) -> None:
    """Threads the CPU engine uses for one host batch below the threshold (default 1)."""
    lib().val_gpu_set_host_cpu_threads(int(threads))


def host_multi_min_bytes(devices: int, pinned: Optional[bool] = None, mean_len: int = 2**64 - 1) -> int:
    """CRC-input bytes below which a *_host_multi batch over `devices`
    distinct GPUs is answered by the CPU engine (decided once per batch);
    pageable input unless `pinned`."""
    if pinned is None:
        return int(lib().val_gpu_host_multi_min_bytes(int(devices)))
    return int(lib().val_gpu_host_multi_min_bytes_ex(int(devices), 1 if pinned else 0, int(mean_len)))


def host_copy_probe(copies: int, nbytes: int, reps: int, pinned: bool = True) -> float:
    """Aggregate GB/s of `copies` concurrent pageable-to-bounce copies through
    the library's own bounce copy (val_gpu_host_copy_probe); no device work."""
    g = ctypes.c_double(0.0)
    _check(lib().val_gpu_host_copy_probe(copies, nbytes, reps, 1 if pinned else 0, ctypes.byref(g)),
           "val_gpu_host_copy_probe")
    return float(g.value)


def set_ragged_min_frames(frames: int) -> None:
    """Mixed-length descriptor batches of at least `frames` frames take the
    device-binned path (-1: VAL_GPU_RAGGED_MIN_FRAMES or the default 4096)."""
    lib().val_gpu_set_ragged_min_frames(int(frames))


def ragged_min_frames() -> int:
    return int(lib().val_gpu_ragged_min_frames())


def scratch_entries(device: int = 0) -> tuple[int, int]:
    """(streams holding library scratch on `device`, LRU evictions so far)."""
    ev = ctypes.c_uint64(0)
    n = lib().val_gpu_scratch_entries(device, ctypes.byref(ev))
    return int(n), int(ev.value)


def cpu_update_state(state: int, data, engine: int = 0) -> int:
    """The library's CPU engine (0 best, 1 slice-by-16, 2 PCLMULQDQ, 3 VPCLMULQDQ)."""
    p, n, keep = _buf(data)
    return int(lib().val_crc32_cpu_update_state(state & 0xFFFFFFFF, p, n, engine))


def cpu_engine() -> int:
    return int(lib().val_crc32_cpu_engine())


def build_flags() -> str:
    """Compile-time switches of the loaded library ("" for a product build)."""
    return lib().val_gpu_build_flags().decode()


def _scalar(fn, *args) -> int:
    """Call a scalar hook and fail loudly if the GPU path failed (the C hooks
    then fall back to the CPU because crc32_func_t has no error channel; this
    Python API has one). Inputs below the provider threshold are answered on
    the CPU by design (last_hook_path() == HOOK_CPU). The check reads the
    calling thread's own record, so other threads' calls do not disturb it."""
    r = int(fn(*args))
    if last_hook_path() == HOOK_FALLBACK:
        raise ValError(VAL_ERR_IO, fn.__name__, "GPU path failed: " + last_error())
    return r


def val_crc32(data) -> int:
    p, n, keep = _buf(data)
    return _scalar(lib().val_crc32, p, n)


def val_crc32_init_state() -> int:
    return int(lib().val_crc32_init_state())


def val_crc32_update_state(state: int, data) -> int:
    p, n, keep = _buf(data)
    return _scalar(lib().val_crc32_update_state, state & 0xFFFFFFFF, p, n)


def val_crc32_finalize_state(state: int) -> int:
    return int(lib().val_crc32_finalize_state(state & 0xFFFFFFFF))


def crc32_provider(seed: int, data) -> int:
    p, n, keep = _buf(data)
    return _scalar(lib().val_gpu_crc32_provider, seed & 0xFFFFFFFF, p, n)


def provider_address() -> int:
    """Address of the C function to store in val_config_t.crc32_provider."""
    return ctypes.cast(lib().val_gpu_crc32_provider, ctypes.c_void_p).value


def crc32_combine(crc_a: int, crc_b: int, len_b: int) -> int:
    return int(lib().val_crc32_combine(crc_a & 0xFFFFFFFF, crc_b & 0xFFFFFFFF, len_b))


def crc32_shift(state: int, nbytes: int) -> int:
    return int(lib().val_crc32_shift(state & 0xFFFFFFFF, nbytes))


def lanes_per_frame(typical_len: int) -> int:
    return int(lib().val_gpu_lanes_per_frame(typical_len))


def set_prefetch(on: int) -> None:
    """Rounds kept in flight ahead of the hashed one: 0, 1, 2, 4, or -1 automatic."""
    _check(lib().val_gpu_set_prefetch(on), "val_gpu_set_prefetch")


def set_geometry(lanes: int = 0, prefetch: int = -1) -> None:
    """Force lanes per frame (0 = automatic) and prefetch (-1 = automatic)."""
    set_lanes_per_frame(lanes)
    set_prefetch(prefetch)


def set_lanes_per_frame(lanes: int) -> None:
    """Force the lanes-per-frame geometry (0 = automatic). Speed only."""
    _check(lib().val_gpu_set_lanes_per_frame(lanes), "val_gpu_set_lanes_per_frame")


# ---- device-resident batches (torch tensors on the GPU) ---------------------
def _dptr(t) -> ctypes.c_void_p:
    if t is None:
        return ctypes.c_void_p(0)
    if not t.is_cuda or not t.is_contiguous():
        raise ValueError("device call needs contiguous GPU tensors")
    return ctypes.c_void_p(t.data_ptr())


def _stream_ptr(stream) -> ctypes.c_void_p:
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def frames(base, *, off=None, length=None, stride: int = 0, flen: int = 0, n: Optional[int] = None,
           out_crc=None, out_hdr=None, len_hint: int = 0, stream=None):
    """Trailer CRC (and optional header_crc) of every frame, device-resident.

    ``base``: uint8 GPU tensor. Descriptor mode: ``off`` (int64) and
    ``length`` (int32) GPU tensors. Strided mode: ``stride``/``flen``/``n``.
    Outputs are int32 GPU tensors holding the uint32 bit patterns.
    Launches on torch's current stream (or ``stream``) and returns at once.
    """
    import torch

    if n is None:
        n = int(off.numel()) if off is not None else 0
    if out_crc is None:
        out_crc = torch.empty(n, dtype=torch.int32, device=base.device)
    st = lib().val_crc32_frames_dev(_dptr(base), _dptr(off), _dptr(length), stride, flen, n, len_hint,
                                    _dptr(out_crc), _dptr(out_hdr), _stream_ptr(stream))
    _check(st, "val_crc32_frames_dev")
    return out_crc


def verify_frames(base, *, off=None, length=None, stride: int = 0, flen: int = 0, n: Optional[int] = None,
                  out_ok=None, nbad=None, out_crc=None, out_hdr=None, len_hint: int = 0, stream=None):
    """RX batch verify. Returns (ok uint8 tensor, nbad int32[1] tensor)."""
    import torch

    if n is None:
        n = int(off.numel()) if off is not None else 0
    dev = base.device
    if out_ok is None:
        out_ok = torch.empty(n, dtype=torch.uint8, device=dev)
    if nbad is None:
        nbad = torch.zeros(1, dtype=torch.int32, device=dev)
    st = lib().val_crc32_verify_frames_dev(_dptr(base), _dptr(off), _dptr(length), stride, flen, n, len_hint,
                                           _dptr(out_ok), _dptr(nbad), _dptr(out_crc), _dptr(out_hdr),
                                           _stream_ptr(stream))
    _check(st, "val_crc32_verify_frames_dev")
    return out_ok, nbad


def verify_frames_ex(base, *, off=None, length=None, stride: int = 0, flen: int = 0, n: Optional[int] = None,
                     out_ok=None, nbad=None, out_crc=None, out_hdr=None, out_pay=None, len_hint: int = 0,
                     stream=None):
    """RX verify with the payload-state by-product (f4). Returns (ok, nbad, pay)
    with pay an int32 tensor of raw zero-init payload registers."""
    import torch

    if n is None:
        n = int(off.numel()) if off is not None else 0
    dev = base.device
    if out_ok is None:
        out_ok = torch.empty(n, dtype=torch.uint8, device=dev)
    if nbad is None:
        nbad = torch.zeros(1, dtype=torch.int32, device=dev)
    if out_pay is None:
        out_pay = torch.empty(n, dtype=torch.int32, device=dev)
    st = lib().val_crc32_verify_frames_ex_dev(_dptr(base), _dptr(off), _dptr(length), stride, flen, n, len_hint,
                                              _dptr(out_ok), _dptr(nbad), _dptr(out_crc), _dptr(out_hdr),
                                              _dptr(out_pay), _stream_ptr(stream))
    _check(st, "val_crc32_verify_frames_ex_dev")
    return out_ok, nbad, out_pay


def region(buf, state_in: int = 0xFFFFFFFF, out=None, stream=None):
    """Raw register after feeding the whole uint8 GPU tensor ``buf``."""
    import torch

    if out is None:
        out = torch.empty(1, dtype=torch.int32, device=buf.device)
    st = lib().val_crc32_region_dev(_dptr(buf), int(buf.numel()), state_in & 0xFFFFFFFF, _dptr(out),
                                    _stream_ptr(stream))
    _check(st, "val_crc32_region_dev")
    return out


# ---- host-memory batches ----------------------------------------------------
class PinnedBuffer:
    """Page-locked host bytes from val_gpu_host_alloc, viewed as a numpy
    uint8 array (`.array`); freed with `.free()` or on garbage collection."""

    def __init__(self, nbytes: int):
        self._lib = lib()
        self._ptr = self._lib.val_gpu_host_alloc(max(1, nbytes))
        if not self._ptr:
            raise ValError(int(VAL_ERR_NO_MEMORY), "val_gpu_host_alloc", last_error())
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array((ctypes.c_uint8 * max(1, nbytes)).from_address(self._ptr))[:nbytes]

    def free(self) -> None:
        if self._ptr:
            self.array = None
            self._lib.val_gpu_host_free(self._ptr)
            self._ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def verify_frames_ex_host(base: np.ndarray, off: Optional[np.ndarray] = None, length: Optional[np.ndarray] = None,
                          stride: int = 0, flen: int = 0, n: Optional[int] = None):
    """Returns (status, ok, nbad, pay uint32 array of payload states)."""
    base = np.ascontiguousarray(base, dtype=np.uint8)
    if off is not None:
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint32)
        n = off.size
    ok = np.zeros(n, dtype=np.uint8)
    pay = np.zeros(n, dtype=np.uint32)
    nbad = ctypes.c_uint32(0)
    st = lib().val_crc32_verify_frames_ex_host(base.ctypes.data, base.size,
                                               off.ctypes.data if off is not None else None,
                                               length.ctypes.data if length is not None else None,
                                               stride, flen, n, ok.ctypes.data, ctypes.byref(nbad), pay.ctypes.data)
    if st not in (VAL_OK, VAL_ERR_CRC):
        _check(st, "val_crc32_verify_frames_ex_host")
    return st, ok, int(nbad.value), pay


def fold_payload_states(state: int, pay_state, pay_len, ok=None) -> tuple[int, int]:
    """Receiver rolling CRC over in-order payload states -> (state, frames folded)."""
    ps = np.ascontiguousarray(pay_state, dtype=np.uint32)
    pl = np.ascontiguousarray(pay_len, dtype=np.uint32)
    okk = np.ascontiguousarray(ok, dtype=np.uint8) if ok is not None else None
    nf = ctypes.c_uint32(0)
    r = lib().val_crc32_fold_payload_states(state & 0xFFFFFFFF, ps.ctypes.data, pl.ctypes.data,
                                            okk.ctypes.data if okk is not None else None, ps.size, ctypes.byref(nf))
    return int(r), int(nf.value)


def fold_payload_states_at(state: int, pay_state, pay_len, file_off, written: int, ok=None) -> tuple[int, int, int]:
    """Receiver rolling CRC with its ordering rule -> (state, written, frames folded)."""
    ps = np.ascontiguousarray(pay_state, dtype=np.uint32)
    pl = np.ascontiguousarray(pay_len, dtype=np.uint32)
    fo = np.ascontiguousarray(file_off, dtype=np.uint64)
    okk = np.ascontiguousarray(ok, dtype=np.uint8) if ok is not None else None
    w = ctypes.c_uint64(written)
    nf = ctypes.c_uint32(0)
    r = lib().val_crc32_fold_payload_states_at(state & 0xFFFFFFFF, ps.ctypes.data, pl.ctypes.data, fo.ctypes.data,
                                               okk.ctypes.data if okk is not None else None, ps.size,
                                               ctypes.byref(w), ctypes.byref(nf))
    return int(r), int(w.value), int(nf.value)


def set_host_chunk_bytes(nbytes: int) -> None:
    """Wire bytes per H2D chunk of the host-memory calls (0 = default 64 MiB)."""
    _check(lib().val_gpu_set_host_chunk_bytes(nbytes), "val_gpu_set_host_chunk_bytes")


def frames_host(base: np.ndarray, off: Optional[np.ndarray] = None, length: Optional[np.ndarray] = None,
                stride: int = 0, flen: int = 0, n: Optional[int] = None, header: bool = False):
    base = np.ascontiguousarray(base, dtype=np.uint8)
    if off is not None:
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint32)
        n = off.size
    crc = np.zeros(n, dtype=np.uint32)
    hdr = np.zeros(n, dtype=np.uint32) if header else None
    st = lib().val_crc32_frames_host(base.ctypes.data, base.size,
                                     off.ctypes.data if off is not None else None,
                                     length.ctypes.data if length is not None else None,
                                     stride, flen, n, crc.ctypes.data,
                                     hdr.ctypes.data if hdr is not None else None)
    _check(st, "val_crc32_frames_host")
    return (crc, hdr) if header else crc


def verify_frames_host(base: np.ndarray, off: Optional[np.ndarray] = None, length: Optional[np.ndarray] = None,
                       stride: int = 0, flen: int = 0, n: Optional[int] = None):
    """Returns (status, ok uint8 array, nbad). status VAL_ERR_CRC on mismatch."""
    base = np.ascontiguousarray(base, dtype=np.uint8)
    if off is not None:
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint32)
        n = off.size
    ok = np.zeros(n, dtype=np.uint8)
    nbad = ctypes.c_uint32(0)
    st = lib().val_crc32_verify_frames_host(base.ctypes.data, base.size,
                                            off.ctypes.data if off is not None else None,
                                            length.ctypes.data if length is not None else None,
                                            stride, flen, n, ok.ctypes.data, ctypes.byref(nbad))
    if st not in (VAL_OK, VAL_ERR_CRC):
        _check(st, "val_crc32_verify_frames_host")
    return st, ok, int(nbad.value)


# ---- several GPUs in one process --------------------------------
def _host_desc(base, off, length):
    base = np.ascontiguousarray(base, dtype=np.uint8)
    if off is not None:
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint32)
    return base, off, length


def frames_host_multi(base: np.ndarray, off: Optional[np.ndarray] = None, length: Optional[np.ndarray] = None,
                      stride: int = 0, flen: int = 0, n: Optional[int] = None, header: bool = False, ndev: int = 0):
    """frames_host split over devices 0..ndev-1 (0: all), one host thread each."""
    base, off, length = _host_desc(base, off, length)
    if off is not None:
        n = off.size
    crc = np.zeros(n, dtype=np.uint32)
    hdr = np.zeros(n, dtype=np.uint32) if header else None
    st = lib().val_crc32_frames_host_multi(base.ctypes.data, base.size, off.ctypes.data if off is not None else None,
                                           length.ctypes.data if length is not None else None, stride, flen, n,
                                           crc.ctypes.data, hdr.ctypes.data if hdr is not None else None, ndev)
    _check(st, "val_crc32_frames_host_multi")
    return (crc, hdr) if header else crc


def verify_frames_host_multi(base: np.ndarray, off: Optional[np.ndarray] = None, length: Optional[np.ndarray] = None,
                             stride: int = 0, flen: int = 0, n: Optional[int] = None, ndev: int = 0):
    """Returns (status, ok uint8 array, nbad); status VAL_ERR_CRC on mismatch."""
    base, off, length = _host_desc(base, off, length)
    if off is not None:
        n = off.size
    ok = np.zeros(n, dtype=np.uint8)
    nbad = ctypes.c_uint32(0)
    st = lib().val_crc32_verify_frames_host_multi(base.ctypes.data, base.size,
                                                  off.ctypes.data if off is not None else None,
                                                  length.ctypes.data if length is not None else None, stride, flen,
                                                  n, ok.ctypes.data, ctypes.byref(nbad), ndev)
    if st not in (VAL_OK, VAL_ERR_CRC):
        _check(st, "val_crc32_verify_frames_host_multi")
    return st, ok, int(nbad.value)


def region_host_multi(data, state_in: int = 0xFFFFFFFF, ndev: int = 0) -> int:
    """Raw register of a host window hashed as ndev byte ranges on ndev GPUs."""
    p, n, keep = _buf(data)
    out = ctypes.c_uint32(0)
    _check(lib().val_crc32_region_host_multi(p, n, state_in & 0xFFFFFFFF, ctypes.byref(out), ndev),
           "val_crc32_region_host_multi")
    return int(out.value)
