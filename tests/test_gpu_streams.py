"""Stream and device handling of the device-resident calls (SURVEY 8(b)
threading: the library must be reentrant from any thread and set its device
per call). Covers what the per-stream scratch design depends on:

* more than 64 streams holding scratch: the least recently used entry is
  evicted after a wait on the completion event bound to its last kernel (not
  a device synchronise, and no HIP call on the stream handle, which may have
  been destroyed), and every result stays exact, including on streams whose
  scratch was evicted and re-created and on new streams after the old ones
  were destroyed;
* hipStreamPerThread from many threads at once, and more than 64 such
  threads over the test: entries are keyed by a per-thread serial that is
  never reused, so a new thread never inherits a live per-thread stream's
  accumulator or queue;
* the device of a call: the stream's device, else the pointer's; the
  caller's HIP device is put back on return.

Reference: src/val_core.c:414-455 (region CRC), :828-834 (frame trailers);
the provider is called under each session's mutex from many threads
(include/val_protocol.h:231-233)."""
import ctypes
import threading

import numpy as np
import pytest

from tests import _oracle, _prng

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

HIP_STREAM_PER_THREAD = 2  # ((hipStream_t)2), hip_runtime_api.h


@pytest.fixture(scope="module")
def vc():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import val_protocol_amd.crc as m

    m.init(0)
    m.set_geometry()
    return m


@pytest.fixture(scope="module")
def hip():
    l = ctypes.CDLL("libamdhip64.so")
    l.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    l.hipStreamSynchronize.restype = ctypes.c_int
    l.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    l.hipStreamCreateWithFlags.restype = ctypes.c_int
    l.hipStreamDestroy.argtypes = [ctypes.c_void_p]
    l.hipStreamDestroy.restype = ctypes.c_int
    return l


def _raw_streams(hip, k):
    """k distinct HIP streams (torch.cuda.Stream() hands out a pool of 32)."""
    out = []
    for _ in range(k):
        h = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(h), 1) == 0  # hipStreamNonBlocking
        out.append((h.value, torch.cuda.ExternalStream(h.value)))
    return out


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


def _ragged(seed, n, lo, hi):
    rng = np.random.default_rng(seed)
    lens = rng.integers(lo, hi + 1, n).astype(np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens.astype(np.uint64) + 4)[:-1]]).astype(np.uint64)
    base = _prng.prng_bytes(seed, int(offs[-1]) + int(lens[-1]) + 4)
    return base, offs, lens


def test_more_streams_than_scratch_entries(vc, hip):
    """80 streams, each with a region window (k_region accumulator) and a
    binned ragged batch (bin scratch): more than the 64 entries a device
    keeps, so the oldest are evicted; then the first streams again (their
    scratch is re-created). Then all 80 are destroyed and 70 new streams
    evict their entries (a destroyed handle's work is finished). Every
    result against the oracle."""
    dev = torch.device("cuda:0")
    vc.set_ragged_min_frames(1)
    data = _prng.prng_bytes(4100, 1 << 20)
    base, offs, lens = _ragged(4101, 600, 0, 9000)
    want_r = _oracle.crc32(data)
    want_f = _oracle.frames(base, offs, lens)
    d_data = torch.from_numpy(data).to(dev)
    d_base = torch.from_numpy(base).to(dev)
    d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    torch.cuda.synchronize()
    _, ev0 = vc.scratch_entries(0)
    def run(streams):
        outs = []
        for _, st in streams:
            r = vc.region(d_data, stream=st)
            c = vc.frames(d_base, off=d_off, length=d_len, stream=st)
            outs.append((r, c))
        torch.cuda.synchronize()
        for r, c in outs:
            assert (int(r.item()) & 0xFFFFFFFF) ^ 0xFFFFFFFF == want_r
            assert np.array_equal(_u32(c), want_f)

    streams = _raw_streams(hip, 80)
    run(streams)
    run(streams[:20])
    entries, ev1 = vc.scratch_entries(0)
    assert entries <= 64
    assert ev1 - ev0 >= 80 + 20 - 64
    for h, _ in streams:
        assert hip.hipStreamDestroy(h) == 0
    fresh = _raw_streams(hip, 70)
    run(fresh)
    entries, ev2 = vc.scratch_entries(0)
    # HIP hands a destroyed stream's handle to a new stream: such a stream
    # finds (inherits) the old entry, whose work is finished; every other new
    # stream evicts one entry
    reused = {h for h, _ in fresh} & {h for h, _ in streams}
    assert entries <= 64 and ev2 - ev1 >= 70 - len(reused)
    for h, _ in fresh:
        assert hip.hipStreamDestroy(h) == 0


def _per_thread_calls(vc, hip, d_data, d_base, d_off, d_len, n, res, k):
    """Region + ragged frames + strided frames on this thread's per-thread
    stream; wait for that stream before the thread exits."""
    l = vc.lib()
    out_r = torch.empty(1, dtype=torch.int32, device=d_data.device)
    out_c = torch.empty(n, dtype=torch.int32, device=d_data.device)
    out_s = torch.empty(64, dtype=torch.int32, device=d_data.device)
    torch.cuda.synchronize()  # the outputs exist before the per-thread stream writes them
    s = ctypes.c_void_p(HIP_STREAM_PER_THREAD)
    st = [
        l.val_crc32_region_dev(ctypes.c_void_p(d_data.data_ptr()), d_data.numel(), 0xFFFFFFFF,
                               ctypes.c_void_p(out_r.data_ptr()), s),
        l.val_crc32_frames_dev(ctypes.c_void_p(d_base.data_ptr()), ctypes.c_void_p(d_off.data_ptr()),
                               ctypes.c_void_p(d_len.data_ptr()), 0, 0, n, 0, ctypes.c_void_p(out_c.data_ptr()),
                               None, s),
        l.val_crc32_frames_dev(ctypes.c_void_p(d_data.data_ptr()), None, None, 16384, 16000, 64, 0,
                               ctypes.c_void_p(out_s.data_ptr()), None, s),
    ]
    st.append(hip.hipStreamSynchronize(s))
    res[k] = (st, out_r, out_c, out_s)


def test_per_thread_streams_concurrent_and_many_threads(vc, hip):
    """8 threads at a time on hipStreamPerThread, 9 waves of threads (72 in
    all, more than the 64 scratch entries): each thread's region, binned
    ragged batch and strided batch against the oracle."""
    dev = torch.device("cuda:0")
    vc.set_ragged_min_frames(1)
    data = _prng.prng_bytes(4200, 1 << 20)
    base, offs, lens = _ragged(4201, 400, 0, 20000)
    want_r = _oracle.crc32(data)
    want_f = _oracle.frames(base, offs, lens)
    want_s = _oracle.frames_strided(data, 16384, 16000, 64)
    d_data = torch.from_numpy(data).to(dev)
    d_base = torch.from_numpy(base).to(dev)
    d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    torch.cuda.synchronize()
    for wave in range(9):
        res = [None] * 8
        th = [threading.Thread(target=_per_thread_calls,
                               args=(vc, hip, d_data, d_base, d_off, d_len, offs.size, res, k)) for k in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        for k, (st, r, c, s) in enumerate(res):
            assert st == [0, 0, 0, 0], (wave, k, st)
            assert (int(r.item()) & 0xFFFFFFFF) ^ 0xFFFFFFFF == want_r, (wave, k)
            assert np.array_equal(_u32(c), want_f), (wave, k)
            assert np.array_equal(_u32(s), want_s), (wave, k)
    entries, _ = vc.scratch_entries(0)
    assert entries <= 64


def test_call_keeps_callers_device(vc):
    """A call on cuda:0 leaves torch's (the thread's HIP) device as it was."""
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    data = _prng.prng_bytes(4300, 100_000)
    r = vc.region(torch.from_numpy(data).to(dev))
    torch.cuda.synchronize()
    assert torch.cuda.current_device() == 0
    assert (int(r.item()) & 0xFFFFFFFF) ^ 0xFFFFFFFF == _oracle.crc32(data)


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2, reason="needs 2 GPUs")
def test_stream_and_pointer_pick_the_device(vc):
    """Thread bound to device 0; tensors and stream on cuda:1: the calls run on
    device 1 (exact results) and the thread's device is still 0 afterwards.
    Without a stream (null), the pointer's device is used."""
    vc.set_device(0)
    torch.cuda.set_device(0)
    d1 = torch.device("cuda:1")
    data = _prng.prng_bytes(4400, 3_000_000)
    base, offs, lens = _ragged(4401, 500, 0, 70000)
    t_data = torch.from_numpy(data).to(d1)
    t_base = torch.from_numpy(base).to(d1)
    t_off = torch.from_numpy(offs.view(np.int64)).to(d1)
    t_len = torch.from_numpy(lens.view(np.int32)).to(d1)
    s1 = torch.cuda.Stream(device=d1)
    torch.cuda.synchronize(d1)
    r = vc.region(t_data, stream=s1)
    c = vc.frames(t_base, off=t_off, length=t_len, stream=s1)
    torch.cuda.synchronize(d1)
    assert torch.cuda.current_device() == 0
    assert (int(r.item()) & 0xFFFFFFFF) ^ 0xFFFFFFFF == _oracle.crc32(data)
    assert np.array_equal(_u32(c), _oracle.frames(base, offs, lens))
    # null stream: the device of the pointer
    out = torch.empty(1, dtype=torch.int32, device=d1)
    st = vc.lib().val_crc32_region_dev(ctypes.c_void_p(t_data.data_ptr()), t_data.numel(), 0xFFFFFFFF,
                                       ctypes.c_void_p(out.data_ptr()), None)
    assert st == 0
    torch.cuda.synchronize(d1)
    assert torch.cuda.current_device() == 0
    assert (int(out.item()) & 0xFFFFFFFF) ^ 0xFFFFFFFF == _oracle.crc32(data)
