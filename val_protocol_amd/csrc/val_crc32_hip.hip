// val_crc32_hip.hip -- host side and C ABI of the VAL CRC-32 integrity path
// on MI355X (gfx950). Kernels: crc_kernels.hpp; device building blocks:
// crc_device.hpp; algorithm and roofline: DESIGN.md; reference call sites per
// entry point: include/val_crc32_gpu.h.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "cpu_crc32.h"
#include "crc_kernels.hpp"
#include "val_crc32_gpu.h"
#include "val_protocol.h"
#include "val_wire.h"

namespace vcrc {

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
// Device scratch of one stream (k_region's accumulator, ragged binning, the
// dynamic-tail queue): a stream's calls are ordered by the stream itself, so
// scratch kept per stream needs no events (an event record + wait per call
// cost ~2.8 us of GPU time on 1 MiB windows, tools/ab_region.py). A stream is
// keyed by its handle, and hipStreamPerThread (one handle naming a different
// real stream on every host thread) by handle and a per-thread serial number
// that is never reused (a std::thread::id is reused once its thread exits,
// and the new thread would then share the old per-thread stream's scratch
// while that stream's kernels may still run). A destroyed stream's handle is
// only reused once its work is done, so inheriting its scratch is safe.
// Callers hold Ctx::mu from acquire through launch.
struct Arena {
    uint8_t *d = nullptr;
    size_t cap = 0;
    bool counts_zero = false;  // counters known to be zero (k_region, launch_ragged re-zero them)
};

struct StreamScratch {
    hipStream_t stream;
    uint64_t owner;     // hipStreamPerThread: the calling thread's serial; else 0
    uint64_t last_use;  // LRU tick (Ctx::scratch_tick)
    // Bound to the dispatch of the last kernel that used this scratch
    // (hipExtLaunchKernelGGL's stop event: no extra queue packet), so
    // eviction waits for exactly that kernel without naming the stream,
    // whose handle may have been destroyed since (HIP calls on a destroyed
    // handle crash) or, for hipStreamPerThread, names another thread's stream.
    hipEvent_t done = nullptr;
    // used by a launch while its stream was capturing a graph: the graph may
    // replay at any time, so the scratch is never evicted
    bool captured = false;
    // a kernel used the scratch without binding `done` (the binning launches
    // before a tracked launch that then failed, or a launch whose capture
    // status could not be queried): not drainable until the next successful
    // tracked launch on the stream, which completes after it
    bool untracked = false;
    Arena region;  // k_region accumulator + arrival count (128 B, zero between calls)
    Arena bin;     // ragged binning: counts, plan, sorted order
    Arena queue;   // k_frames dynamic tail {head, exits} (zero between calls)
    Arena tail;    // k_frames in-launch tail pieces: {register, arrivals} per tail frame (zero between calls)
};
// Streams with scratch per device; beyond this the least recently used entry
// is evicted (a program that keeps creating streams would otherwise grow the
// list without bound).
constexpr size_t kMaxStreamScratch = 64;
std::atomic<uint64_t> g_thread_serial{0};
thread_local uint64_t t_thread_serial = 0;  // 0: not assigned yet
uint64_t thread_serial()
{
    if (!t_thread_serial) t_thread_serial = g_thread_serial.fetch_add(1) + 1;
    return t_thread_serial;
}

// One context per HIP device: streams, constant blob, staging and scratch.
// A process may drive any number of devices; each host thread works on the
// device it is bound to (val_gpu_set_device / val_gpu_init), else on the
// process default (the first device initialised). hipSetDevice is per host
// thread, so every entry point sets it before touching HIP.
struct Ctx {
    std::recursive_mutex mu;
    std::vector<StreamScratch *> scratch;  // per stream handle
    uint64_t scratch_tick = 0;
    uint64_t scratch_evictions = 0;
    int device = -1;
    int cus = 0;
    hipStream_t stream = nullptr;
    uint8_t *d_stage = nullptr;   // host-API staging (frames, region input)
    size_t d_stage_cap = 0;
    uint8_t *d_small = nullptr;   // descriptors / outputs for host APIs
    size_t d_small_cap = 0;
    uint32_t *d_consts = nullptr; // constant blob (tables, gap and merge maps)
    // host-API pipeline: frames go H2D in chunks on `copy` while the previous
    // chunk is hashed on `stream` (two device slots; two pinned bounce
    // buffers for pageable inputs)
    hipStream_t copy = nullptr;
    hipEvent_t h2d_done[2] = {}, kern_done[2] = {};
    uint8_t *d_slot[2] = {};
    size_t d_slot_cap[2] = {};
    uint8_t *h_bounce[2] = {};
    size_t h_bounce_cap[2] = {};
    uint8_t *h_out = nullptr;     // pinned landing buffer of the host APIs' D2H results
    size_t h_out_cap = 0;
};

constexpr int kMaxDevices = 64;
std::mutex g_ctx_mu;                     // guards g_ctxs creation / teardown
std::atomic<Ctx *> g_ctxs[kMaxDevices] = {};  // published once initialised
std::atomic<int> g_default_dev{-1};      // first device initialised in this process
thread_local int t_dev = -1;             // device the calling thread is bound to
thread_local std::string t_err;

val_status_t fail(val_status_t st, const char *what, hipError_t e = hipSuccess)
{
    char buf[256];
    if (e != hipSuccess)
        snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
    else
        snprintf(buf, sizeof buf, "%s", what);
    t_err = buf;
    return st;
}

#define VCRC_HIP(call, what)                                   \
    do {                                                       \
        hipError_t e_ = (call);                                \
        if (e_ != hipSuccess) return fail(VAL_ERR_IO, what, e_); \
    } while (0)

void ctx_free(Ctx &c);

val_status_t ctx_init(Ctx &c, int device)
{
    VCRC_HIP(hipSetDevice(device), "hipSetDevice");
    hipDeviceProp_t prop;
    VCRC_HIP(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return fail(VAL_ERR_IO, "val_gpu_init: device is not gfx950");
    c.device = device;
    VCRC_HIP(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking), "hipStreamCreate");
    VCRC_HIP(hipStreamCreateWithFlags(&c.copy, hipStreamNonBlocking), "hipStreamCreate(copy)");
    for (int i = 0; i < 2; i++) {
        VCRC_HIP(hipEventCreateWithFlags(&c.h2d_done[i], hipEventDisableTiming), "hipEventCreate");
        VCRC_HIP(hipEventCreateWithFlags(&c.kern_done[i], hipEventDisableTiming), "hipEventCreate");
    }
    {
        std::vector<uint32_t> blob(kConstWords);
        fill_const_blob(blob.data());
        VCRC_HIP(hipMalloc((void **)&c.d_consts, blob.size() * 4u), "hipMalloc(consts)");
        VCRC_HIP(hipMemcpy(c.d_consts, blob.data(), blob.size() * 4u, hipMemcpyHostToDevice), "H2D consts");
    }
    c.cus = prop.multiProcessorCount;
    return VAL_OK;
}

// Context of `device`, created on first use.
val_status_t get_ctx(int device, Ctx **out)
{
    if (device >= 0 && device < kMaxDevices) {  // fast path: no HIP call once initialised
        Ctx *c = g_ctxs[device].load(std::memory_order_acquire);
        if (c) {
            *out = c;
            return VAL_OK;
        }
    }
    int count = 0;
    hipError_t e = hipGetDeviceCount(&count);
    if (e != hipSuccess || count <= 0) return fail(VAL_ERR_IO, "val_gpu_init: no HIP device", e);
    if (device < 0 || device >= count || device >= kMaxDevices)
        return fail(VAL_ERR_INVALID_ARG, "val_gpu_init: device index out of range");
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    if (!g_ctxs[device].load(std::memory_order_acquire)) {
        Ctx *c = new Ctx;
        val_status_t st = ctx_init(*c, device);
        if (st != VAL_OK) {
            ctx_free(*c);
            delete c;
            return st;
        }
        g_ctxs[device].store(c, std::memory_order_release);
        int none = -1;
        g_default_dev.compare_exchange_strong(none, device);
    }
    *out = g_ctxs[device].load(std::memory_order_acquire);
    return VAL_OK;
}

// The caller's HIP device, put back when an entry point returns: the library
// sets the device it works on (hipSetDevice is per host thread), and must
// not leave the caller's thread (e.g. torch's) on another one.
struct DeviceScope {
    int saved = -1;
    DeviceScope()
    {
        if (hipGetDevice(&saved) != hipSuccess) {
            (void)hipGetLastError();
            saved = -1;
        }
    }
    ~DeviceScope()
    {
        int now = -1;
        if (saved >= 0 && hipGetDevice(&now) == hipSuccess && now != saved) (void)hipSetDevice(saved);
    }
};

val_status_t ctx_on(int d, Ctx **out)
{
    val_status_t st = get_ctx(d, out);
    if (st != VAL_OK) return st;
    VCRC_HIP(hipSetDevice(d), "hipSetDevice");  // device is per host thread in HIP
    return VAL_OK;
}

// The calling thread's context (its bound device, else the process default,
// else device 0), with the thread's HIP device set to it. Host-memory calls.
val_status_t cur(Ctx **out)
{
    int d = t_dev >= 0 ? t_dev : g_default_dev.load(std::memory_order_relaxed);
    if (d < 0) d = 0;
    return ctx_on(d, out);
}

// Context of a device-resident call: the device of its stream, else the
// device `ptr` (the frame or window base) lives on, else the thread's
// device as in cur(). A cuda:1 tensor on a cuda:1 stream therefore runs on
// device 1 whatever device the calling thread was bound to.
val_status_t cur_dev(void *stream, const void *ptr, Ctx **out)
{
    const hipStream_t s = (hipStream_t)stream;
    int d = -1;
    if (s && s != hipStreamPerThread && s != hipStreamLegacy) {
        hipDevice_t dev = -1;
        if (hipStreamGetDevice(s, &dev) == hipSuccess) d = (int)dev;
        else (void)hipGetLastError();
    }
    if (d < 0 && ptr) {
        hipPointerAttribute_t attr;
        if (hipPointerGetAttributes(&attr, ptr) == hipSuccess && attr.type == hipMemoryTypeDevice) d = attr.device;
        else (void)hipGetLastError();
    }
    return d >= 0 ? ctx_on(d, out) : cur(out);
}

bool valid_lanes(uint32_t g) { return g == 1 || g == 2 || g == 4 || g == 8 || g == 16 || g == 32 || g == 64; }

std::atomic<uint32_t> g_forced_lanes{0};
std::atomic<int> g_forced_prefetch{-1};

uint32_t env_u32(const char *name)
{
    const char *e = getenv(name);
    return e ? (uint32_t)atoi(e) : 0u;
}

// Lanes forced by val_gpu_set_lanes_per_frame or VAL_GPU_LANES_PER_FRAME (0 = none).
uint32_t forced_lanes()
{
    static const uint32_t env_g = env_u32("VAL_GPU_LANES_PER_FRAME");
    const uint32_t forced = g_forced_lanes.load(std::memory_order_relaxed);
    if (valid_lanes(forced)) return forced;
    return valid_lanes(env_g) ? env_g : 0u;
}

// Lanes that share one frame (G) in uniform batches, by length: the measured
// best of the current kernels (profiles/r03_length_sweep.log, strided 3 GB
// batches): 2 below 1 KiB, 4 below 2 KiB, 8 below 48 KiB,
// 16 above. G = 8 from 2 KiB gained 3-5% over G = 4 on 2-4 KiB frames and
// 5% on u4200d (profiles/r03_ab_geom_short.log). The ragged path keeps its
// length classes (kClassLanes), whose buckets are rounds of their class.
uint32_t lanes_per_frame(uint32_t len)
{
    const uint32_t f = forced_lanes();
    if (f) return f;
    return len < 1024u ? 2u : len < 2048u ? 4u : len < 49152u ? 8u : 16u;
}

// G for a uniform batch of n frames of len bytes: the class's G, doubled while
// the batch would leave more than half of the machine's waves idle (a small
// window spreads each frame over more lanes, so its serial chain is shorter),
// up to one wave per frame and at most one 64-B unit per lane per round. The
// doubling only acts on batches of fewer groups than half the machine's waves
// (one pass of the grid); large batches keep the class's measured G. Capping
// it at 16 cost small windows of long frames 1.5-2.5x (256 x 64 KiB: 103 ->
// 41 us per call; 256 x 16 KiB: 34 -> 20 us; profiles/r02_ab_lanes_cap.log).
uint32_t lanes_for_batch(const Ctx &c, uint32_t len, uint64_t n)
{
    uint32_t G = lanes_per_frame(len);
    if (forced_lanes()) return G;
    const uint64_t waves = (uint64_t)c.cus * kWavesPerBlock;
    const uint64_t units = len ? (len + kUnit - 1) / kUnit : 1u;
    const uint32_t cap = 64u;
    while (G < cap && 2u * G <= units && (n + 64 / G - 1) / (64 / G) * 2u <= waves) G *= 2;
    return G;
}

// 0, 1, 2, 4: copy-and-refill depths; -2, -3: in-place rings (G = 2 and 4 only)
bool valid_prefetch(int d) { return d == 0 || d == 1 || d == 2 || d == 4 || d == -2 || d == -3; }

// Prefetch depth forced by val_gpu_set_prefetch or VAL_GPU_PREFETCH (-1 = none).
int forced_prefetch()
{
    static const int env_p = getenv("VAL_GPU_PREFETCH") ? atoi(getenv("VAL_GPU_PREFETCH")) : -1;
    const int forced = g_forced_prefetch.load(std::memory_order_relaxed);
    if (forced != -1) return forced;
    return valid_prefetch(env_p) ? env_p : -1;
}

// Rounds kept in flight ahead of the one being hashed: 1 unless forced
// (launch_uniform_g turns the automatic 1 into the in-place rings at G = 2, 4).
// Measured on MI355X (profiles/r01_small_batches.log): issuing every round up
// front (2 or 4 deep) lost 5-15% even on one-pass batches such as cfg2, since
// the whole batch's requests then land before any wave can start hashing.
int prefetch_depth()
{
    const int forced = forced_prefetch();
    return forced != -1 ? forced : 1;
}

StreamScratch &scratch_for(Ctx &c, hipStream_t s);
template <typename K, typename... Args>
hipError_t launch_tracked(StreamScratch *x, K kernel, dim3 grid, dim3 block, hipStream_t s, Args... args);

// one_pass: every wave hashes at most one frame group (windows, cfg2): round
// 0's units by dword loads (k_frames C0; crc_kernels.hpp load_unit0).
// x: the stream scratch the launch uses (the dynamic-tail queue), else null.
template <int G>
hipError_t launch_uniform_g(int pf, dim3 grid, hipStream_t s, const FrameParams &p, bool one_pass, StreamScratch *x,
                             uint32_t len)
{
    const dim3 b(kBlock);
    if (p.out_pay) return launch_tracked(x, k_frames<G, 1, true>, grid, b, s, p);  // payload states: default depth only
// A/B builds: one-pass launches' round loop. Rings measured no better on
// cfg2 (two deep +0.6% back to back, -3.7% single launch; three deep -7%) and
// equal on 64-4,096-frame windows (profiles/r04_ab_ring_prefetch_one_pass.log).
#ifndef VCRC_C0_PF
#define VCRC_C0_PF 1
#endif
    if (pf == 1 && one_pass) return launch_tracked(x, k_frames<G, (G == 2 || G == 4) ? VCRC_C0_PF : 1, false, true>, grid, b, s, p);
    // Multi-pass short frames hash each round in its registers and refill them
    // in place (a ring of -pf rounds, crc_kernels.hpp hash_frame BURST):
    // profiles/r04_ab_ring_prefetch.log, same box against the copy-and-refill
    // PF = 1 loop: G = 2 three deep u600d +4.2% (two deep +1.8%); G = 4 two
    // deep u1100d +1.5-1.8%, s1100 0%, u2000d -0.3 to -0.6% (three deep -0.7 to
    // -3%), so 4 lanes take the ring below 1,600 B (R <= 7) only.
#ifndef VCRC_RING_G2
#define VCRC_RING_G2 -3
#endif
#ifndef VCRC_RING_G4
#define VCRC_RING_G4 -2
#endif
    if (pf == 1 && forced_prefetch() == -1) pf = G == 2 ? VCRC_RING_G2 : (G == 4 && len < 1600u) ? VCRC_RING_G4 : 1;
    if constexpr (G == 2 || G == 4) {
        if (pf == -3) return launch_tracked(x, k_frames<G, -3, false>, grid, b, s, p);
        if (pf == -2) return launch_tracked(x, k_frames<G, -2, false>, grid, b, s, p);
    }
    switch (pf) {
    case 0: return launch_tracked(x, k_frames<G, 0, false>, grid, b, s, p);
    case 2: return launch_tracked(x, k_frames<G, 2, false>, grid, b, s, p);
    case 4: return launch_tracked(x, k_frames<G, 4, false>, grid, b, s, p);
    default: return launch_tracked(x, k_frames<G, 1, false>, grid, b, s, p);
    }
}

val_status_t arena_acquire(Arena &a, size_t bytes, hipStream_t s, uint8_t **out);

// Dynamic tail of long uniform launches (k_frames): VAL_GPU_DYNAMIC_TAIL=0/1.
// A launch takes it when it is long enough for the queue to pay: 8 or 16
// lanes per frame from 1.45 MiB of frames per wave (about 6 GB at 4,096
// waves), 2 or 4 lanes from 8 group rounds. Shorter launches measured faster
// static, once the exits were counted per workgroup (same box, back to back,
// profiles/r06_ab_dyn_tail_rules.log): 64 KiB frames 4 / 5 rounds -2.5 /
// -0.6% with the queue, 6 / 7 rounds +0.5 / +1.0%; 16,400-B frames 6 / 8
// rounds -3.7 / -1.6%, 12 / 16 rounds +0.5 / +1.6%; 4,200-B frames (8 lanes,
// 34 KiB groups) 4 / 8 / 12 rounds -8 / -5 / -3.6%; 1,100-B and 2,000-B frames
// at 4 rounds -5% and -3.9%, 600-B and 1,100-B frames at 8 rounds +3.6% and
// +3.2%.
#ifndef VCRC_DYN_MIN_WAVE_BYTES
#define VCRC_DYN_MIN_WAVE_BYTES 1520000u
#endif
#ifndef VCRC_DYN_MIN_ROUNDS_SHORT
#define VCRC_DYN_MIN_ROUNDS_SHORT 8
#endif
#ifndef VCRC_DYN_TAIL_DEFAULT
#define VCRC_DYN_TAIL_DEFAULT 1
#endif
bool dyn_tail_enabled()
{
    static const bool on = getenv("VAL_GPU_DYNAMIC_TAIL") ? atoi(getenv("VAL_GPU_DYNAMIC_TAIL")) != 0
                                                         : VCRC_DYN_TAIL_DEFAULT != 0;
    return on;
}

// Small batches of long frames go to k_frames_split (one workgroup per frame,
// its chunks hashed by 16 waves at once) when that takes fewer memory rounds
// per wave than one wave per frame: ceil(n / CUs) passes of about three
// round-times each (a chunk round, the fold, the next frame's start) against
// ceil(units / 64) rounds. Measured (profiles/r02_ab_split.log): 256 x 64 KiB
// 41 -> 18 us per call, 256 x 8 KiB 21.5 -> 16 us, equal at 1024 x 64 KiB,
// slower at 2048 x 64 KiB and 512 x 16 KiB (the rule keeps those off it).
// Payload states and forced geometries keep the frames kernels.
// VAL_GPU_SPLIT=0 disables it.
bool split_enabled()
{
#ifdef VCRC_NO_SPLIT  // A/B builds only
    return false;
#endif
    static const bool on = !(getenv("VAL_GPU_SPLIT") && atoi(getenv("VAL_GPU_SPLIT")) == 0);
    return on;
}

bool use_split(const Ctx &c, const FrameParams &p, uint32_t len)
{
    if (!split_enabled() || p.out_pay || forced_lanes() || forced_prefetch() != -1 || len < 8192u) return false;
    const uint64_t waves = (uint64_t)c.cus * kWavesPerBlock;
    if ((uint64_t)p.n * 2u > waves) return false;
    const uint64_t rounds = ((uint64_t)len / kUnit + 1u + 63u) / 64u;  // at one wave per frame
    const uint64_t passes = ((uint64_t)p.n + c.cus - 1u) / (uint64_t)c.cus;
    return passes * 3u <= rounds;
}

val_status_t launch_split(const Ctx &c, FrameParams &p, uint32_t len, hipStream_t s)
{
    p.consts = c.d_consts;
    // W = 2^k0 >= 1 KiB with a typical frame in at most 16 chunks (one group)
    uint32_t k0 = 10;
    while (((uint64_t)kWavesPerBlock << k0) < (uint64_t)len && k0 < 31) k0++;
    const dim3 grid((unsigned)std::min<uint64_t>(p.n, (uint64_t)c.cus));
    hipLaunchKernelGGL(k_frames_split, grid, dim3(kBlock), 0, s, p, k0);
    VCRC_HIP(hipGetLastError(), "k_frames_split launch");
    return VAL_OK;
}

val_status_t launch_uniform_one(const Ctx &c, FrameParams &p, uint32_t G, uint32_t len, hipStream_t s)
{
    p.consts = c.d_consts;
// A/B builds: multi-pass G = 2/4 batches on 512-thread workgroups (8 waves
// per CU, up to 256 VGPRs: 185 used) with a ring of -VCRC_W8_PF rounds, so a
// 1,100-B group's rounds are all in flight at entry. 10-24% slower than 16
// waves with the 2/3-rings (u1100d -23%, s1100 -18%, u600d -11%, u2000d -10%;
// profiles/r04_ab_eight_waves_deep_ring.log): the table chains need the waves.
#ifndef VCRC_W8_PF
#define VCRC_W8_PF 0
#endif
    const bool w8 = VCRC_W8_PF != 0 && (G == 2 || G == 4) && !p.out_pay && forced_prefetch() == -1 &&
                    (uint64_t)p.n > (uint64_t)c.cus * 16u * (64u / G);  // more than one pass at 16 waves per CU
    const uint32_t wpb = w8 ? 8u : (uint32_t)kWavesPerBlock;
    const uint64_t groups_per_block = (uint64_t)wpb * (64 / G);
    uint64_t blocks = (p.n + groups_per_block - 1) / groups_per_block;
    blocks = std::max<uint64_t>(1, std::min<uint64_t>(blocks, (uint64_t)c.cus));  // persistent, 1 per CU (LDS)
    const dim3 grid((unsigned)blocks);
    const int pf = prefetch_depth();
    // Dynamic tail for long launches: the last half of the group rounds come
    // from a queue (k_frames). Groups of >= 128 KiB (strided) or 192 KiB
    // (descriptors) pull from one word: 4,096 waves over 128 KiB groups is
    // about 48 dequeues/us at 6 TB/s, under the ~88/us one word serves, and
    // one word evens the end out better than partitions (cfg3 -1.5%, cfg4 -3.7%
    // with 64). Groups under 128 KiB pull from 64 partitions: descriptor groups
    // from 16 KiB (round 2: u4200d +4%, u1100d +6%; with one word they lost up to 2x),
    // strided ones from 32 KiB (s4200 +3%; s1100's 17.6 KiB groups -3%);
    // descriptor groups of 128-192 KiB stay static below 16 rounds (u16400d
    // -1% either way: profiles/r02_ab_dynparts.log) and take one word above.
    // Which launches are long enough for any queue: VCRC_DYN_MIN_WAVE_BYTES above.
    const uint64_t rounds = ((uint64_t)p.n + 64 / G - 1) / (64 / G) / (blocks * wpb);
    p.qhead = nullptr;
    const uint64_t group_bytes = (uint64_t)(64 / G) * len;
#ifndef VCRC_DYN_MIN_GROUP  // A/B builds may override: one-word minimum group bytes, strided / descriptor batches
#define VCRC_DYN_MIN_GROUP (128u << 10)
#endif
#ifndef VCRC_DYN_MIN_GROUP_DESC
#define VCRC_DYN_MIN_GROUP_DESC (192u << 10)
#endif
#ifndef VCRC_DYN_MIN_GROUP_PARTS  // partitioned queue minimum group bytes, strided / descriptor batches
#define VCRC_DYN_MIN_GROUP_PARTS (32u << 10)
#endif
#ifndef VCRC_DYN_MIN_GROUP_PARTS_DESC
#define VCRC_DYN_MIN_GROUP_PARTS_DESC (16u << 10)
#endif
    // Descriptor groups of 128-192 KiB take the one-word queue only from 16
    // rounds on: cfg3's layout through descriptors (32 rounds) +3.0%, 3 GB of
    // 16,400-B frames (6 rounds) -2.8% with it (profiles/r06_ab_desc_dyn_tail.log).
#ifndef VCRC_DYN_DESC_LONG_ROUNDS
#define VCRC_DYN_DESC_LONG_ROUNDS 16
#endif
    const bool one_word = group_bytes >= (p.off ? (rounds >= VCRC_DYN_DESC_LONG_ROUNDS ? VCRC_DYN_MIN_GROUP
                                                                                       : VCRC_DYN_MIN_GROUP_DESC)
                                                : VCRC_DYN_MIN_GROUP);
    const bool parts =
        group_bytes >= (p.off ? VCRC_DYN_MIN_GROUP_PARTS_DESC : VCRC_DYN_MIN_GROUP_PARTS) && group_bytes < VCRC_DYN_MIN_GROUP;
    // the queue's scratch may be dropped by scratch_for (another stream's call)
    // unless the lock is held until the kernel is launched
    Ctx &cm = const_cast<Ctx &>(c);
    std::lock_guard<std::recursive_mutex> lk(cm.mu);
    StreamScratch *used = nullptr;
    if (p.tail_n) {  // in-launch tail pieces (launch_uniform): a zeroed accumulator pair per tail frame
        used = &scratch_for(cm, s);
        Arena &a = used->tail;
        uint8_t *q = nullptr;
        const size_t bytes = (size_t)p.tail_n * 8u;
        val_status_t st = arena_acquire(a, bytes, s, &q);
        if (st != VAL_OK) return st;
        if (!a.counts_zero) VCRC_HIP(hipMemsetAsync(q, 0, a.cap, s), "hipMemsetAsync(tail)");
        a.counts_zero = false;  // set again once the launch is queued (its last pieces re-zero the pairs)
        p.tail_acc = reinterpret_cast<uint32_t *>(q);
    }
    const bool long_enough = G >= 8 ? rounds * group_bytes >= (uint64_t)VCRC_DYN_MIN_WAVE_BYTES
                                    : rounds >= VCRC_DYN_MIN_ROUNDS_SHORT;
    if (dyn_tail_enabled() && long_enough && (one_word || parts)) {
        if (!used) used = &scratch_for(cm, s);
        Arena &a = used->queue;
        uint8_t *q = nullptr;
        val_status_t st = arena_acquire(a, kDynQueueBytes, s, &q);
        if (st != VAL_OK) return st;
        if (!a.counts_zero) VCRC_HIP(hipMemsetAsync(q, 0, kDynQueueBytes, s), "hipMemsetAsync(queue)");
        a.counts_zero = true;  // the last wave out re-zeroes it
        p.qhead = reinterpret_cast<uint32_t *>(q);
        p.qparts = one_word ? 1u : kDynParts;
#ifndef VCRC_DYN_DIV
#define VCRC_DYN_DIV 2
#endif
        p.static_rounds = (uint32_t)(VCRC_DYN_DIV == 1 ? 1u : rounds - std::max<uint64_t>(1, rounds / VCRC_DYN_DIV));
    }
    const bool one_pass = ((uint64_t)p.n + 64 / G - 1) / (64 / G) <= (uint64_t)grid.x * wpb;
    hipError_t e = hipSuccess;
    if (w8) {
        if (G == 2) e = launch_tracked(used, k_frames<2, (VCRC_W8_PF < 0 ? VCRC_W8_PF : -2), false, false, 512>, grid, dim3(512), s, p);
        else e = launch_tracked(used, k_frames<4, (VCRC_W8_PF < 0 ? VCRC_W8_PF : -2), false, false, 512>, grid, dim3(512), s, p);
        VCRC_HIP(e, "k_frames launch");
        return VAL_OK;
    }
    switch (G) {
    case 1: e = launch_uniform_g<1>(pf, grid, s, p, one_pass, used, len); break;
    case 2: e = launch_uniform_g<2>(pf, grid, s, p, one_pass, used, len); break;
    case 4: e = launch_uniform_g<4>(pf, grid, s, p, one_pass, used, len); break;
    case 8: e = launch_uniform_g<8>(pf, grid, s, p, one_pass, used, len); break;
    case 16: e = launch_uniform_g<16>(pf, grid, s, p, one_pass, used, len); break;
    case 32: e = launch_uniform_g<32>(pf, grid, s, p, one_pass, used, len); break;
    case 64: e = launch_uniform_g<64>(pf, grid, s, p, one_pass, used, len); break;
    default: return fail(VAL_ERR_INVALID_ARG, "bad lanes-per-frame");
    }
    if (p.tail_n && e == hipSuccess) used->tail.counts_zero = true;
    VCRC_HIP(e, "k_frames launch");
    return VAL_OK;
}

// In-launch tail pieces (crc_kernels.hpp tail_pieces): the frames past the
// last full wave-round, cut into pieces of W = 2^k0 bytes and hashed by the
// oldest waves as one extra frame group each, instead of a second launch.
// W = 1 KiB (one round at 16 lanes: the extra work per wave stays under what
// the oldest waves gain on the youngest), doubled while the piece groups
// outnumber the waves. Kernels with G = 8 or 16 at the default depth carry
// the path; frames of at least 8 KiB use it. VAL_GPU_TAIL_PIECES=0 or
// val_gpu_set_tail_pieces(0) keeps the second launch (A/B).
std::atomic<int> g_tail_pieces{-1};  // -1: VAL_GPU_TAIL_PIECES (unset = on); 0 / 1: val_gpu_set_tail_pieces
std::atomic<uint64_t> g_tail_piece_launches{0};
bool tail_pieces_enabled()
{
    const int v = g_tail_pieces.load(std::memory_order_relaxed);
    if (v >= 0) return v != 0;
    static const bool on = !(getenv("VAL_GPU_TAIL_PIECES") && atoi(getenv("VAL_GPU_TAIL_PIECES")) == 0);
    return on;
}

// log2 of the piece bytes for this tail, or 0 when the path does not apply.
uint32_t tail_piece_k0(const Ctx &c, const FrameParams &p, uint32_t G, uint32_t len, uint64_t n_tail)
{
    if (!tail_pieces_enabled() || p.out_pay || (G != 8 && G != 16) || len < 8192u || n_tail == 0 ||
        forced_prefetch() != -1)
        return 0;
    for (uint32_t k0 = kPieceK0Min; k0 <= 16; k0++) {
        const uint64_t units = n_tail * (((uint64_t)len + (1u << k0) - 1) >> k0);
        if ((units + 64 / G - 1) / (64 / G) <= (uint64_t)c.cus * kWavesPerBlock) return k0;
    }
    return 0;
}

// Persistent waves take whole frame groups, so a launch lasts
// ceil(groups / waves) group-times: 131,113 frames of 64 KiB at G = 16 are
// 8.002 wave-rounds, the last one 99.8% idle. The frames of a partial last
// round are re-cut with more lanes per frame (up to 64) into a second launch
// on the same stream, so the tail costs about G / G_tail of a group-time.
val_status_t launch_uniform(const Ctx &c, FrameParams &p, uint32_t G, uint32_t len, hipStream_t s)
{
    const uint64_t per = 64 / G, groups = (p.n + per - 1) / per;
    const uint64_t waves = (uint64_t)c.cus * kWavesPerBlock;
    const uint64_t full = groups / waves;
    uint32_t Gt = G;
    const uint64_t n_main = full * waves * per, n_tail = p.n - std::min<uint64_t>(p.n, n_main);
    if (full > 0 && n_tail > 0)
        while (Gt < 64 && (n_tail + 64 / (2 * Gt) - 1) / (64 / (2 * Gt)) <= waves) Gt *= 2;
    if (Gt == G) return launch_uniform_one(c, p, G, len, s);
    if (const uint32_t k0 = tail_piece_k0(c, p, G, len, n_tail)) {
        FrameParams m = p;
        m.n = (uint32_t)n_main;
        m.tail_n = (uint32_t)n_tail;
        m.tail_k0 = k0;
        m.tail_units = (uint32_t)(((uint64_t)len + (1u << k0) - 1) >> k0);
        if (!p.off) {
            m.last_len = p.flen;  // frame n_main - 1 is a full one
            m.tail_last_len = p.last_len;
        }
        const val_status_t st = launch_uniform_one(c, m, G, len, s);
        if (st == VAL_OK) g_tail_piece_launches.fetch_add(1, std::memory_order_relaxed);
        return st;
    }
    FrameParams m = p, t = p;
    m.n = (uint32_t)n_main;
    t.n = (uint32_t)n_tail;
    if (p.off) {
        t.off = p.off + n_main;
        t.len = p.len + n_main;
    } else {
        m.last_len = p.flen;
        t.base = p.base + n_main * p.stride;
    }
    t.seed0 = p.seed_rest;  // frame 0 is in the main part
    if (p.out_crc) t.out_crc = p.out_crc + n_main;
    if (p.out_hdr) t.out_hdr = p.out_hdr + n_main;
    if (p.out_ok) t.out_ok = p.out_ok + n_main;
    if (p.out_pay) t.out_pay = p.out_pay + n_main;
    val_status_t st = launch_uniform_one(c, m, G, len, s);
    if (st != VAL_OK) return st;
    // a tail of a few long frames (cfg4: 41 x 64 KiB after 8 full rounds) is a
    // small batch of its own: one workgroup per frame when that is faster
    const uint32_t tl = t.off ? len : std::max(t.flen, t.last_len);
    if (use_split(c, t, tl)) return launch_split(c, t, tl, s);
    return launch_uniform_one(c, t, Gt, tl, s);
}

void arena_free(Arena &a);

void scratch_free(StreamScratch *x)
{
    arena_free(x->region);
    arena_free(x->queue);
    arena_free(x->tail);
    arena_free(x->bin);
    if (x->done) (void)hipEventDestroy(x->done);
    delete x;
}

// Wait until no kernel still uses x's scratch: its last kernel's completion
// event. False when the entry cannot be drained (graph capture) or the wait
// failed; the caller then evicts another entry.
bool scratch_drain(StreamScratch *x)
{
    if (x->captured || x->untracked || !x->done) return false;
    if (hipEventSynchronize(x->done) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return true;
}

// Scratch of stream s (the calling thread's per-thread stream for
// hipStreamPerThread). A full list evicts its least recently used entry
// after draining it (scratch_drain); if no entry can be drained (every other
// one is captured in a graph), the list grows past its cap.
StreamScratch &scratch_for(Ctx &c, hipStream_t s)
{
    const uint64_t who = s == hipStreamPerThread ? thread_serial() : 0u;
    const uint64_t tick = ++c.scratch_tick;
    for (StreamScratch *x : c.scratch)
        if (x->stream == s && x->owner == who) {
            x->last_use = tick;
            return *x;
        }
    if (c.scratch.size() >= kMaxStreamScratch) {
        std::vector<StreamScratch *> by_age(c.scratch);
        std::sort(by_age.begin(), by_age.end(),
                  [](const StreamScratch *a, const StreamScratch *b) { return a->last_use < b->last_use; });
        for (StreamScratch *x : by_age) {
            if (!scratch_drain(x)) continue;
            c.scratch.erase(std::find(c.scratch.begin(), c.scratch.end(), x));
            scratch_free(x);
            c.scratch_evictions++;
            break;
        }
    }
    StreamScratch *x = new StreamScratch{s, who, tick};
    if (hipEventCreateWithFlags(&x->done, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        x->done = nullptr;  // never drained: never evicted
    }
    c.scratch.push_back(x);
    return *x;
}

// Launch a kernel that uses x's scratch, binding x's completion event to the
// dispatch. While s is capturing a graph the kernel is launched plainly and
// the entry is kept for good (the graph owns that use of the scratch). When
// the capture status cannot be queried (e.g. the legacy stream while another
// stream captures) the launch is plain and the entry is held only until the
// next tracked launch succeeds; a failed tracked launch holds it the same way.
template <typename K, typename... Args>
hipError_t launch_tracked(StreamScratch *x, K kernel, dim3 grid, dim3 block, hipStream_t s, Args... args)
{
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    bool unknown = false;
    if (x && hipStreamIsCapturing(s, &cap) != hipSuccess) {
        (void)hipGetLastError();
        unknown = true;
    }
    if (x && !unknown && cap == hipStreamCaptureStatusNone && x->done) {
        hipExtLaunchKernelGGL(kernel, grid, block, 0, s, nullptr, x->done, 0u, args...);
        const hipError_t e = hipGetLastError();
        x->untracked = e != hipSuccess;  // on failure `done` names an older dispatch
        return e;
    }
    if (x && unknown) x->untracked = true;
    else if (x) x->captured = true;
    hipLaunchKernelGGL(kernel, grid, block, 0, s, args...);
    return hipGetLastError();
}


// Scratch of at least `bytes` for stream s. Growing waits for the stream's
// earlier kernels, which may still use the old block.
val_status_t arena_acquire(Arena &a, size_t bytes, hipStream_t s, uint8_t **out)
{
    if (a.cap < bytes) {
        VCRC_HIP(hipStreamSynchronize(s), "hipStreamSynchronize(scratch)");
        if (a.d) (void)hipFree(a.d);
        a.d = nullptr;
        a.cap = 0;
        a.counts_zero = false;
        const size_t sz = std::max<size_t>(bytes, 1u << 20);
        hipError_t e = hipMalloc((void **)&a.d, sz);
        if (e != hipSuccess) return fail(VAL_ERR_NO_MEMORY, "hipMalloc(scratch)", e);
        a.cap = sz;
    }
    *out = a.d;
    return VAL_OK;
}

void arena_free(Arena &a)
{
    if (a.d) (void)hipFree(a.d);
    a = Arena{};
}

// Ragged descriptor batch: counting-sort by length on the device, then one
// grouped launch planned by bytes per length class (no host synchronisation).
val_status_t launch_ragged(Ctx &c, FrameParams &p, hipStream_t s)
{
    const uint32_t n = p.n;
    const uint32_t nbin = std::max(1u, std::min(1024u, (n + 2047u) / 2048u));
    const uint32_t chunk = (n + nbin - 1) / nbin;
    // scratch: heads[kQueueParts][16] u32 | gcount[kBuckets] u32 | ctab[16] u32 | blockoff[nbin][kBuckets] u32 |
    //          order[n] u32. gcount is zero between batches (k_frames_ragged re-zeroes it once
    //          k_bin_scatter has read it); heads are zeroed by k_bin_scatter.
    const size_t sz_heads = (size_t)kQueueParts * 64u, sz_gcount = (size_t)kBuckets * 4u;
    const size_t total = sz_heads + sz_gcount + 64u + (size_t)nbin * kBuckets * 4u + (size_t)n * 4u;
    std::lock_guard<std::recursive_mutex> lk(c.mu);
    StreamScratch &ss = scratch_for(c, s);
    Arena &a = ss.bin;
    uint8_t *scratch = nullptr;
    val_status_t st = arena_acquire(a, total, s, &scratch);
    if (st != VAL_OK) return st;
    uint32_t *heads = reinterpret_cast<uint32_t *>(scratch);
    uint32_t *gcount = heads + sz_heads / 4u;
    uint32_t *ctab = gcount + kBuckets;
    uint32_t *blockoff = ctab + 16;
    uint32_t *order = blockoff + (size_t)nbin * kBuckets;
    // New scratch, or a batch whose launches failed part-way: zero the counts.
    hipError_t e = a.counts_zero ? hipSuccess : hipMemsetAsync(gcount, 0, sz_gcount, s);
    a.counts_zero = false;
    if (e == hipSuccess) {
        ss.untracked = true;  // the binning launches are not bound to `done`; the tracked launch clears it
        hipLaunchKernelGGL(k_bin_count, dim3(nbin), dim3(kBinThreads), 0, s, p.len, n, chunk, gcount, blockoff);
        hipLaunchKernelGGL(k_bin_scatter, dim3(nbin), dim3(kBinThreads), 0, s, p.len, n, chunk, gcount, blockoff, ctab,
                           heads, order);
        p.consts = c.d_consts;
        p.order = order;
        p.plan = ctab;
        p.heads = heads;
        p.bin_counts = gcount;
        // persistent: enough waves for the items, at most one workgroup per CU
        const uint64_t max_items = (n + 3u) / 4u + kClasses;  // every class packs >= 4 frames per item
        const unsigned blocks = (unsigned)std::max<uint64_t>(
            1, std::min<uint64_t>((uint64_t)c.cus, (max_items + kWavesPerBlock - 1) / kWavesPerBlock));
        // the ragged kernel is the last of the three on the stream to use the scratch
        if (p.out_pay) e = launch_tracked(&ss, k_frames_ragged<1, true>, dim3(blocks), dim3(kBlock), s, p);
        else if (forced_prefetch() == 0) e = launch_tracked(&ss, k_frames_ragged<0, false>, dim3(blocks), dim3(kBlock), s, p);
// A/B builds: the ragged kernel's round loop (1 = copy and refill, -2 / -3 =
// rings). The rings lost 9-11% on cfg5 and the class-2 mix and 2-3% on 600 and
// 1,100-B frames through the ragged path (profiles/r04_ab_ring_prefetch_ragged.log).
#ifndef VCRC_RAGGED_PF
#define VCRC_RAGGED_PF 1
#endif
        else e = launch_tracked(&ss, k_frames_ragged<VCRC_RAGGED_PF, false>, dim3(blocks), dim3(kBlock), s, p);
        a.counts_zero = e == hipSuccess;
    }
    if (e != hipSuccess) return fail(VAL_ERR_IO, "ragged frames launch", e);
    return VAL_OK;
}

// typical_len == 0 with descriptors means "lengths unknown or mixed": bin them,
// unless the batch is too small to fill the machine once (binning is four
// launches; a small window runs uniform at 16 lanes per frame instead).
// val_gpu_set_ragged_min_frames, else VAL_GPU_RAGGED_MIN_FRAMES (read once),
// overrides the threshold (tests pin the binned path on small batches).
constexpr uint32_t kRaggedMinFrames = 4096;
std::atomic<int64_t> g_ragged_min{-1};  // -1: from the environment, else the default

// A size knob from the environment, read once: a malformed value (e.g. "1M")
// is reported once on stderr and the built-in default is used.
int64_t env_size(const char *name)
{
    const char *e = getenv(name);
    if (!e || !*e) return -1;
    char *end = nullptr;
    const long long v = strtoll(e, &end, 0);
    if (end == e || *end != '\0' || v < 0) {
        fprintf(stderr, "val_crc32_gpu: ignoring %s=\"%s\" (not a non-negative integer); using the default\n", name, e);
        return -1;
    }
    return (int64_t)v;
}

uint32_t ragged_min_frames()
{
    const int64_t v = g_ragged_min.load(std::memory_order_relaxed);
    if (v >= 0) return (uint32_t)std::min<int64_t>(v, UINT32_MAX);
    static const int64_t env = env_size("VAL_GPU_RAGGED_MIN_FRAMES");
    return env >= 0 ? (uint32_t)std::min<int64_t>(env, UINT32_MAX) : kRaggedMinFrames;
}

val_status_t launch_frames(Ctx &c, FrameParams &p, uint32_t typical_len, hipStream_t s)
{
    if (p.n == 0) return VAL_OK;
    if (p.off && typical_len == 0 && !forced_lanes() && p.n >= ragged_min_frames()) return launch_ragged(c, p, s);
    const uint32_t len = typical_len ? typical_len : 16384u;
    const uint32_t longest = !p.off ? std::max(p.flen, p.last_len) : len;
    if (use_split(c, p, longest)) return launch_split(c, p, longest, s);
    return launch_uniform(c, p, lanes_for_batch(c, len, p.n), len, s);
}

// NULL selects the HIP default (null) stream, as in every HIP API.
hipStream_t pick_stream(void *stream) { return (hipStream_t)stream; }

// Region geometry: up to 64 KiB one K1 "frame" at 64 lanes (one launch, no
// fold); longer windows go to k_region with chunks of W = 2^k0 >= 4 KiB,
// doubling until there are at most 4,096 chunks (one per wave of the
// machine; 256 MiB = 4,096 chunks of 64 KiB = 16 rounds per lane).
constexpr uint64_t kRegionOneFrame = 8u << 10;  // one 64-lane frame of <= 2 rounds; k_region is faster above (profiles/r02_region_latency.log: 16 KiB 8.9 us as one frame, 8.2 us in k_region)
constexpr uint64_t kRegionMaxPiece = (uint64_t)kRegionMaxChunks << 31;  // W <= 2^31: longer windows chain pieces
void region_geometry(uint64_t len, uint64_t *W, uint32_t *k0, uint32_t *C)
{
    uint32_t k = 12;
    while (((uint64_t)kRegionMaxChunks << k) < len) k++;
    *k0 = k;
    *W = (uint64_t)1 << k;
    *C = (uint32_t)((len + *W - 1) >> k);
}

val_status_t region_dev(Ctx &c, const uint8_t *d_ptr, uint64_t len, uint32_t state_in, uint32_t *d_out, hipStream_t s,
                        const uint32_t *seed_dev = nullptr)
{
    if (len <= kRegionOneFrame && !seed_dev) {
        FrameParams p{};
        p.base = d_ptr;
        p.stride = len ? len : 1;
        p.flen = (uint32_t)len;
        p.last_len = (uint32_t)len;
        p.n = 1;
        p.seed0 = p.seed_rest = state_in;
        p.xorout = 0;
        p.out_crc = d_out;
        return launch_frames(c, p, (uint32_t)len, s);
    }
    // Beyond 2^43 bytes: pieces chained through the device state (each piece
    // reads the previous one's result as its seed). VAL_GPU_REGION_MAX_PIECE
    // lowers the piece size (tests exercise the chaining).
    static const uint64_t env_piece = getenv("VAL_GPU_REGION_MAX_PIECE") ? strtoull(getenv("VAL_GPU_REGION_MAX_PIECE"), nullptr, 0) : 0;
    const uint64_t piece = env_piece > kRegionOneFrame ? std::min(env_piece, kRegionMaxPiece) : kRegionMaxPiece;
    if (len > piece) {
        val_status_t st = VAL_OK;
        for (uint64_t o = 0; o < len && st == VAL_OK; o += piece)
            st = region_dev(c, d_ptr + o, std::min(piece, len - o), state_in, d_out, s, o ? d_out : seed_dev);
        return st;
    }
    std::lock_guard<std::recursive_mutex> lk(c.mu);
    StreamScratch &ss = scratch_for(c, s);
    Arena &a = ss.region;
    uint8_t *scratch = nullptr;
    val_status_t st = arena_acquire(a, 128, s, &scratch);
    if (st != VAL_OK) return st;
    hipError_t e = a.counts_zero ? hipSuccess : hipMemsetAsync(scratch, 0, 128, s);
    a.counts_zero = false;
    if (e == hipSuccess) {
        RegionParams rp{};
        rp.base = d_ptr;
        rp.len = len;
        region_geometry(len, &rp.W, &rp.k0, &rp.C);
        rp.nwg = (rp.C + kWavesPerBlock - 1) / kWavesPerBlock;
        rp.seed = state_in;
        rp.seed_dev = seed_dev;
        rp.out = d_out;
        rp.acc = reinterpret_cast<uint32_t *>(scratch);
        rp.consts = c.d_consts;
        e = launch_tracked(&ss, k_region, dim3(rp.nwg), dim3(kBlock), s, rp);
        a.counts_zero = e == hipSuccess;  // the last workgroup re-zeroes the scratch
    }
    if (e != hipSuccess) return fail(VAL_ERR_IO, "k_region launch", e);
    return VAL_OK;
}

val_status_t grow(uint8_t **buf, size_t *cap, size_t need)
{
    if (*cap >= need) return VAL_OK;
    if (*buf) (void)hipFree(*buf);
    *buf = nullptr;
    *cap = 0;
    size_t sz = std::max<size_t>(need, 1u << 20);
    hipError_t e = hipMalloc((void **)buf, sz);
    if (e != hipSuccess) return fail(VAL_ERR_NO_MEMORY, "hipMalloc(staging)", e);
    *cap = sz;
    return VAL_OK;
}

std::atomic<size_t> g_host_chunk{0};
constexpr size_t kDefaultHostChunk = 64u << 20;

size_t host_chunk_bytes()
{
    const size_t c = g_host_chunk.load(std::memory_order_relaxed);
    return c ? c : kDefaultHostChunk;
}

// Pinned (page-locked) host memory is copied by DMA straight from the
// caller's buffer; pageable memory goes through pinned bounce buffers.
bool is_pinned(const void *p)
{
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return attr.type == hipMemoryTypeHost;
}

// memcpy into a pinned bounce chunk with up to 8 host threads, one per 4
// MiB. Concurrent copies (one per device in the *_host_multi calls) share
// the process's CPU affinity set: the threads of all copies in flight never
// exceed it (8 devices x 8 threads would be 64 threads on a 16-core share).
// The budget is the affinity set capped by the cgroup CPU quota: a GPU box
// shows every CPU of the machine in the affinity set (256) but its quota pays
// for one GPU's share (16).
unsigned cgroup_cpu_quota()
{
    unsigned q = 0;
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {  // cgroup v2: "<quota> <period>" or "max <period>"
        char a[32] = {0};
        double per = 0;
        if (fscanf(f, "%31s %lf", a, &per) == 2 && strcmp(a, "max") != 0 && per > 0) {
            const double v = atof(a) / per;
            if (v > 0) q = (unsigned)std::max(1.0, v + 0.999);
        }
        fclose(f);
        return q;
    }
    FILE *fq = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r");  // cgroup v1
    FILE *fp = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r");
    double quota = -1, per = 0;
    if (fq && fp && fscanf(fq, "%lf", &quota) == 1 && fscanf(fp, "%lf", &per) == 1 && quota > 0 && per > 0)
        q = (unsigned)std::max(1.0, quota / per + 0.999);
    if (fq) fclose(fq);
    if (fp) fclose(fp);
    return q;
}

unsigned host_cpu_budget()
{
    static const unsigned n = [] {
        unsigned a = std::max(1u, std::thread::hardware_concurrency());
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof set, &set) == 0) a = (unsigned)std::max(1, CPU_COUNT(&set));
        const unsigned q = cgroup_cpu_quota();
        return q ? std::min(a, q) : a;
    }();
    return n;
}

// Threads one copy of n bytes gets when `concurrent` copies run at once.
uint32_t copy_threads(uint64_t n, uint32_t concurrent)
{
    const uint64_t share = std::max<uint64_t>(1, host_cpu_budget() / std::max<uint32_t>(1, concurrent));
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>({8u, share, (n + (4u << 20) - 1) / (4u << 20)}));
}

std::atomic<uint32_t> g_copies_in_flight{0};

void parallel_copy(uint8_t *dst, const uint8_t *src, size_t n)
{
    const uint32_t concurrent = g_copies_in_flight.fetch_add(1) + 1;
    const size_t nt = copy_threads(n, concurrent);
    if (nt <= 1) {
        memcpy(dst, src, n);
    } else {
        std::vector<std::thread> th;
        const size_t per = (n + nt - 1) / nt;
        for (size_t t = 1; t < nt; t++) {
            const size_t lo = t * per, hi = std::min(n, lo + per);
            if (lo >= hi) continue;
            try {
                th.emplace_back([=] { memcpy(dst + lo, src + lo, hi - lo); });
            } catch (...) {  // no thread: the calling thread copies this piece
                memcpy(dst + lo, src + lo, hi - lo);
            }
        }
        memcpy(dst, src, std::min(n, per));  // the calling thread takes the first piece
        for (auto &x : th) x.join();
    }
    g_copies_in_flight.fetch_sub(1);
}

val_status_t grow_pinned(uint8_t **buf, size_t *cap, size_t need)
{
    if (*cap >= need) return VAL_OK;
    if (*buf) (void)hipHostFree(*buf);
    *buf = nullptr;
    *cap = 0;
    hipError_t e = hipHostMalloc((void **)buf, need, hipHostMallocDefault);
    if (e != hipSuccess) return fail(VAL_ERR_NO_MEMORY, "hipHostMalloc(bounce)", e);
    *cap = need;
    return VAL_OK;
}

// Pageable host -> device, through the two pinned bounce buffers on stream s.
// hipMemcpyAsync straight from pageable memory is not used anywhere: on this
// ROCm it let the next kernel on a non-blocking stream read part of a > 64 KiB
// copy before it landed (~7% wrong CRCs on 64-70 KiB provider calls, none
// through pinned staging; tests/test_gpu_dropin.py::test_provider_stress_*).
val_status_t h2d_staged(Ctx &c, uint8_t *dst, const uint8_t *src, size_t bytes, hipStream_t s)
{
    if (!bytes) return VAL_OK;
    const size_t chunk = std::min(bytes, host_chunk_bytes());
    val_status_t st;
    for (int k = 0; k < 2; k++)
        if ((st = grow_pinned(&c.h_bounce[k], &c.h_bounce_cap[k], chunk)) != VAL_OK) return st;
    int k = 0;
    for (size_t o = 0; o < bytes; o += chunk, k ^= 1) {
        const size_t nb = std::min(chunk, bytes - o);
        VCRC_HIP(hipEventSynchronize(c.h2d_done[k]), "hipEventSynchronize");  // bounce k drained
        parallel_copy(c.h_bounce[k], src + o, nb);
        VCRC_HIP(hipMemcpyAsync(dst + o, c.h_bounce[k], nb, hipMemcpyHostToDevice, s), "H2D");
        VCRC_HIP(hipEventRecord(c.h2d_done[k], s), "hipEventRecord");
    }
    return VAL_OK;
}

// Wait for a short host-path call (scalar hooks, zero-copy windows): poll
// hipStreamQuery for up to kSpinNs, about 1 us less per call than blocking at
// once (provider 16 B: 19.0 -> 17.7 us; profiles/r02_ab_provider_spin.log),
// then block in hipStreamSynchronize, so a long call does not burn the core
// while the caller holds VAL's session mutex. The chunked pipeline, whose
// calls last milliseconds, blocks from the start.
constexpr int64_t kSpinNs = 50000;
hipError_t host_wait(hipStream_t s)
{
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t e;
    while ((e = hipStreamQuery(s)) == hipErrorNotReady) {
        if (std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count() > kSpinNs)
            return hipStreamSynchronize(s);
    }
    return e;
}

// Host pointer -> region state on the calling thread's device (the scalar
// hooks and each shard of region_host_multi).
val_status_t region_host(const void *data, size_t len, uint32_t state_in, uint32_t *state_out)
{
    DeviceScope ds;
    Ctx *cp = nullptr;
    val_status_t st = cur(&cp);
    if (st != VAL_OK) return st;
    Ctx &c = *cp;
    std::lock_guard<std::recursive_mutex> lk(c.mu);
    if ((st = grow(&c.d_stage, &c.d_stage_cap, len ? len : 1)) != VAL_OK) return st;
    if ((st = grow_pinned(&c.h_out, &c.h_out_cap, 64)) != VAL_OK) return st;
    hipStream_t s = c.stream;
    // The kernel writes the state straight into pinned host memory (no D2H
    // command). Inputs up to kZeroCopy are read by the kernel from a pinned
    // bounce buffer in place (zero-copy over PCIe, no H2D command); longer
    // ones are staged into HBM first.
    constexpr size_t kZeroCopy = 16u << 10;
    const uint8_t *src = c.d_stage;
    if (len && len <= kZeroCopy) {
        if ((st = grow_pinned(&c.h_bounce[0], &c.h_bounce_cap[0], len)) != VAL_OK) return st;
        VCRC_HIP(hipEventSynchronize(c.h2d_done[0]), "hipEventSynchronize");
        memcpy(c.h_bounce[0], data, len);
        src = c.h_bounce[0];
    } else if ((st = h2d_staged(c, c.d_stage, static_cast<const uint8_t *>(data), len, s)) != VAL_OK) {
        return st;
    }
    uint32_t *h_state = reinterpret_cast<uint32_t *>(c.h_out);
    if ((st = region_dev(c, src, len, state_in, h_state, s)) != VAL_OK) return st;
    VCRC_HIP(hipEventRecord(c.h2d_done[0], s), "hipEventRecord");  // the kernel may read bounce 0
    VCRC_HIP(host_wait(s), "hipStreamQuery");
    memcpy(state_out, h_state, 4);
    return VAL_OK;
}

// ---- the scalar hooks: CPU below a size threshold, GPU above -----------------
// crc32_func_t has no error channel (reference include/val_protocol.h:163-166)
// and the reference calls it under the session mutex on every frame
// (src/val_core.c:721-836, :884-1045) with host memory in and one CRC out.
// A GPU call costs a launch and a completion wait (~18 us) plus the bytes
// over PCIe, while the reference's byte loop costs ~1.7 us per KiB: below the
// provider threshold the three scalar hooks answer with this library's own
// CPU engine (cpu_crc32.c: carry-less-multiply folding, slice-by-16 where the
// CPU lacks it), so installing the provider never makes VAL slower. At and
// above the threshold they run on the GPU. The threshold is measured
// (tools/provider_latency.py); VAL_GPU_PROVIDER_MIN_BYTES
// or val_gpu_set_provider_min_bytes overrides it (0 = always the GPU: the GPU
// test suite sets it, so every hook it checks ran on the GPU).
// Failure policy: when the GPU path fails (no device, a HIP error), the hooks
// compute the CRC with the same CPU engine and count it
// (val_gpu_cpu_fallback_count); VAL_GPU_CPU_FALLBACK=0 or
// val_gpu_set_cpu_fallback(0) makes a failed hook abort instead. Nothing else
// has a CPU path: batch calls return VAL_ERR_IO.
std::atomic<uint64_t> g_cpu_fallbacks{0};
// Hook calls answered below the provider threshold: counted on every VAL frame
// by every session thread, so the count is sharded over cache lines (one per
// thread, round-robin) and summed on read. One shared counter made concurrent
// sessions take turns on its line: 16-B calls cost 24 ns on one thread and
// 373 ns each on eight (the provider's whole cost, oracle/provider_bench.c).
struct alignas(64) CountShard {
    std::atomic<uint64_t> v{0};
};
constexpr int kCountShards = 64;
CountShard g_cpu_small[kCountShards];
std::atomic<uint32_t> g_next_shard{0};
thread_local int t_count_shard = -1;
inline void count_small()
{
    if (t_count_shard < 0) t_count_shard = (int)(g_next_shard.fetch_add(1, std::memory_order_relaxed) % kCountShards);
    g_cpu_small[t_count_shard].v.fetch_add(1, std::memory_order_relaxed);
}
uint64_t cpu_small_total()
{
    uint64_t t = 0;
    for (const CountShard &c : g_cpu_small) t += c.v.load(std::memory_order_relaxed);
    return t;
}
std::atomic<int> g_cpu_fallback_on{-1};  // -1: from the environment
std::atomic<int64_t> g_provider_min{-1};  // -1: from the environment, else the default
thread_local int t_hook_path = VAL_GPU_HOOK_NONE;

#ifndef VCRC_PROVIDER_MIN_BYTES  // measured crossover, DESIGN.md section 1
#define VCRC_PROVIDER_MIN_BYTES (256u << 20)
#endif

uint64_t provider_min_bytes()
{
    const int64_t v = g_provider_min.load(std::memory_order_relaxed);
    if (v >= 0) return (uint64_t)v;
    static const int64_t env = env_size("VAL_GPU_PROVIDER_MIN_BYTES");
    return env >= 0 ? (uint64_t)env : (uint64_t)VCRC_PROVIDER_MIN_BYTES;
}

bool cpu_fallback_enabled()
{
    const int v = g_cpu_fallback_on.load(std::memory_order_relaxed);
    if (v >= 0) return v != 0;
    const char *e = getenv("VAL_GPU_CPU_FALLBACK");
    return !(e && e[0] == '0');
}

[[noreturn]] void die(const char *fn)
{
    fprintf(stderr, "val_crc32_gpu: %s failed on the GPU path: %s (CPU fallback disabled)\n", fn, t_err.c_str());
    abort();
}

uint32_t scalar_state(const char *fn, uint32_t state, const void *data, size_t len)
{
    uint32_t out = 0;
    if (len && !data) die(fn);  // the reference dereferences it too
    if ((uint64_t)len < provider_min_bytes()) {
        t_hook_path = VAL_GPU_HOOK_CPU;
        count_small();
        return vcrc_cpu_update(state, data, len);
    }
    if (region_host(data, len, state, &out) == VAL_OK) {
        t_hook_path = VAL_GPU_HOOK_GPU;
        return out;
    }
    if (!cpu_fallback_enabled()) die(fn);
    t_hook_path = VAL_GPU_HOOK_FALLBACK;
    if (g_cpu_fallbacks.fetch_add(1, std::memory_order_relaxed) == 0)
        fprintf(stderr, "val_crc32_gpu: %s: GPU path failed (%s); CRC computed on the CPU (counted)\n", fn,
                t_err.c_str());
    return vcrc_cpu_update(state, data, len);
}

// Small host windows (<= 256 KiB of wire span): one launch and no copy
// commands. Frames and descriptors sit in one pinned buffer (the caller's, if
// its frames are pinned already) that the kernel reads in place over PCIe,
// and the results are written straight into pinned host memory; the mismatch
// count is taken from the ok flags on the host. A 16-frame 1 KiB window cost
// ~64 us through the chunked pipeline (a descriptor copy, a memset, a frames
// copy, a launch, a results copy).
constexpr uint64_t kHostZeroCopy = 256u << 10;
val_status_t frames_host_small(Ctx &c, const uint8_t *base, uint64_t lo, uint64_t hi, const uint64_t *off,
                               const uint32_t *len, uint64_t stride, uint32_t flen, uint32_t n, int verify,
                               uint32_t hint, uint32_t *crc, uint32_t *hdr, uint8_t *ok, uint32_t *nbad, uint32_t *pay)
{
    const size_t span = (size_t)(hi - lo), desc = off ? (size_t)n * 12u : 0u;
    const size_t span_al = (span + 15u) & ~(size_t)15u;
    const bool pinned = is_pinned(base);
    val_status_t st;
    if ((st = grow_pinned(&c.h_bounce[0], &c.h_bounce_cap[0], (pinned ? 0u : span_al) + desc + 16u)) != VAL_OK)
        return st;
    if ((st = grow_pinned(&c.h_out, &c.h_out_cap, (size_t)n * 13u + 16u)) != VAL_OK) return st;
    VCRC_HIP(hipEventSynchronize(c.h2d_done[0]), "hipEventSynchronize");  // nothing still reads bounce 0
    uint8_t *b = c.h_bounce[0];
    const uint8_t *frames = base + lo;
    if (!pinned) {
        memcpy(b, base + lo, span);
        frames = b;
    }
    uint64_t *h_off = nullptr;
    uint32_t *h_len = nullptr;
    if (off) {  // rebased: frame i sits at frames + h_off[i]
        h_off = reinterpret_cast<uint64_t *>(b + (pinned ? 0u : span_al));
        h_len = reinterpret_cast<uint32_t *>(h_off + n);
        for (uint32_t i = 0; i < n; i++) h_off[i] = off[i] - lo;
        memcpy(h_len, len, (size_t)n * 4u);
    }
    uint32_t *h_crc = reinterpret_cast<uint32_t *>(c.h_out);
    uint32_t *h_hdr = h_crc + n;
    uint32_t *h_pay = h_hdr + n;
    uint8_t *h_ok = reinterpret_cast<uint8_t *>(h_pay + n + 4);
    FrameParams p{};
    p.base = frames;
    p.off = h_off;
    p.len = h_len;
    p.stride = stride;
    p.flen = flen;
    p.last_len = flen;
    p.n = n;
    p.seed0 = p.seed_rest = 0xFFFFFFFFu;
    p.xorout = 0xFFFFFFFFu;
    p.out_crc = crc ? h_crc : nullptr;
    p.out_hdr = hdr ? h_hdr : nullptr;
    p.verify = verify ? 1u : 0u;
    p.out_ok = (ok || nbad) ? h_ok : nullptr;
    p.nbad = nullptr;
    p.out_pay = pay ? h_pay : nullptr;
    hipStream_t s = c.stream;
    if ((st = launch_frames(c, p, hint, s)) != VAL_OK) return st;
    VCRC_HIP(hipEventRecord(c.h2d_done[0], s), "hipEventRecord");  // the kernel reads bounce 0
    VCRC_HIP(host_wait(s), "hipStreamQuery");
    if (crc) memcpy(crc, h_crc, (size_t)n * 4u);
    if (hdr) memcpy(hdr, h_hdr, (size_t)n * 4u);
    if (pay) memcpy(pay, h_pay, (size_t)n * 4u);
    if (ok) memcpy(ok, h_ok, n);
    if (nbad) {
        uint32_t bad = 0;
        for (uint32_t i = 0; i < n; i++) bad += h_ok[i] == 0;
        *nbad = verify ? bad : 0u;
    }
    return VAL_OK;
}

// ---- host-memory batches below the measured crossover: the CPU engine --------
// A host batch on the GPU pays a launch, a completion wait and PCIe for every
// byte (51 GiB/s at best), while one core of the CPU
// engine folds 41-47 GB/s from DRAM: below the crossover (DESIGN.md section 1,
// tools/host_crossover.py) the *_frames_host calls answer with the CPU engine
// on the calling thread (val_gpu_set_host_cpu_threads adds helper threads),
// with the same outputs as the kernels: trailer CRC, header_crc, verify flags
// and count, payload states. Counted (val_gpu_cpu_batch_count);
// VAL_GPU_HOST_BATCH_MIN_BYTES or val_gpu_set_host_batch_min_bytes moves the
// threshold (0 = always the GPU: the GPU test suite sets it).
// The crossover depends on the frame size: the CPU engine folds long frames
// from DRAM about twice as fast as 1 KiB frames, so at one CPU thread the GPU
// path (pageable) wins from about 32 MiB of 1 KiB frames but only past 64 MiB
// of 16-64 KiB frames (profiles/r04_host_crossover.jsonl, r05_host_crossover_
// fine.jsonl). The default is therefore chosen by the batch's mean CRC input
// per frame; a value set by the environment or the setter applies to all.
#ifndef VCRC_HOST_BATCH_MIN_BYTES  // measured crossover at one CPU thread, frames of >= 4 KiB
#define VCRC_HOST_BATCH_MIN_BYTES (64u << 20)
#endif
#ifndef VCRC_HOST_BATCH_MIN_BYTES_SHORT  // the same for a mean frame under 4 KiB
#define VCRC_HOST_BATCH_MIN_BYTES_SHORT (32u << 20)
#endif
constexpr uint64_t kShortFrameMean = 4096;
std::atomic<int64_t> g_host_batch_min{-1};  // -1: from the environment, else the default
std::atomic<uint32_t> g_host_cpu_threads{1};
std::atomic<uint64_t> g_cpu_batches{0};

uint64_t host_batch_min_bytes(uint64_t mean_len = UINT64_MAX)
{
    const int64_t v = g_host_batch_min.load(std::memory_order_relaxed);
    if (v >= 0) return (uint64_t)v;
    static const int64_t env = env_size("VAL_GPU_HOST_BATCH_MIN_BYTES");
    if (env >= 0) return (uint64_t)env;
    return mean_len < kShortFrameMean ? (uint64_t)VCRC_HOST_BATCH_MIN_BYTES_SHORT : (uint64_t)VCRC_HOST_BATCH_MIN_BYTES;
}

std::vector<uint32_t> shard_cuts(uint32_t n, const uint32_t *len, uint32_t world);

// Frames [i0, i1) of a host batch on the CPU engine (outputs as frames_host).
uint32_t cpu_frames_range(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride,
                          uint32_t flen, uint32_t i0, uint32_t i1, int verify, uint32_t *crc, uint32_t *hdr,
                          uint8_t *ok, uint32_t *pay)
{
    uint32_t bad = 0;
    for (uint32_t i = i0; i < i1; i++) {
        const uint8_t *p = base + (off ? off[i] : (uint64_t)i * stride);
        const uint32_t L = len ? len[i] : flen;
        const uint32_t c = vcrc_cpu_update(0xFFFFFFFFu, p, L) ^ 0xFFFFFFFFu;
        if (crc) crc[i] = c;
        if (hdr) hdr[i] = vcrc_cpu_update(0xFFFFFFFFu, p, std::min<uint32_t>(L, 8u)) ^ 0xFFFFFFFFu;
        if (pay) {
            // the kernels' payload by-product: the register of the payload from
            // zero, after the 8-B header and the 8-B offset when flags say so
            const uint32_t pre = L >= 8 ? ((p[1] & VAL_DATA_OFFSET_PRESENT) ? 16u : 8u) : UINT32_MAX;
            pay[i] = (L >= 8 && L >= pre) ? vcrc_cpu_update(0u, p + pre, L - pre) : 0u;
        }
        if (verify) {
            const uint32_t t = (uint32_t)p[L] | (uint32_t)p[L + 1] << 8 | (uint32_t)p[L + 2] << 16 |
                               (uint32_t)p[L + 3] << 24;
            if (ok) ok[i] = c == t ? 1u : 0u;
            bad += c != t;
        }
    }
    return bad;
}

// The whole batch on the calling thread plus helper threads (contiguous
// frame ranges balanced by bytes, as the multi-GPU split).
// Helper threads only for batches of at least 4 MiB per thread: a thread
// start costs more than a small window's whole CRC. The thread count is
// val_gpu_set_host_cpu_threads capped by the process's CPU budget (affinity
// and cgroup quota). A helper thread that cannot be started leaves its range
// to the calling thread (the C entry points must not throw).
uint32_t cpu_frames(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t stride, uint32_t flen,
                    uint32_t n, uint64_t total, int verify, uint32_t *crc, uint32_t *hdr, uint8_t *ok, uint32_t *pay)
{
    g_cpu_batches.fetch_add(1, std::memory_order_relaxed);
    const uint64_t by_size = std::max<uint64_t>(1, total >> 22);
    const uint32_t nt = (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>({(uint64_t)g_host_cpu_threads.load(), (uint64_t)host_cpu_budget(), by_size,
                               (uint64_t)std::max(n, 1u)}));
    if (nt == 1) return cpu_frames_range(base, off, len, stride, flen, 0, n, verify, crc, hdr, ok, pay);
    const std::vector<uint32_t> cut = shard_cuts(n, len, nt);
    std::vector<uint32_t> bad(nt, 0);
    std::vector<std::thread> th;
    uint32_t started = 1;  // ranges [1, started) run on helper threads
    for (; started < nt; started++) {
        const uint32_t t = started;
        try {
            th.emplace_back([&, t] {
                bad[t] = cpu_frames_range(base, off, len, stride, flen, cut[t], cut[t + 1], verify, crc, hdr, ok, pay);
            });
        } catch (...) {
            break;
        }
    }
    bad[0] = cpu_frames_range(base, off, len, stride, flen, cut[0], cut[1], verify, crc, hdr, ok, pay);
    for (uint32_t t = started; t < nt; t++)
        bad[t] = cpu_frames_range(base, off, len, stride, flen, cut[t], cut[t + 1], verify, crc, hdr, ok, pay);
    for (auto &x : th) x.join();
    uint32_t nbad = 0;
    for (uint32_t b : bad) nbad += b;
    return nbad;
}

// Host-memory batches on the calling thread's device: descriptors H2D once,
// then frames in chunks of whole frames (<= host_chunk_bytes of wire span
// each) through two device slots: chunk c's H2D on the copy stream overlaps
// chunk c-1's kernel on the compute stream; the outputs come back D2H once at
// the end. Descriptor batches are chunked when their offsets are
// non-decreasing (a packed stream); otherwise the whole span is one chunk.
// route_cpu == false: the caller (frames_host_multi) already chose the GPU for
// the whole batch, so this shard skips the single-GPU crossover.
val_status_t frames_host(const uint8_t *base, uint64_t base_len, const uint64_t *off, const uint32_t *len,
                         uint64_t stride, uint32_t flen, uint32_t n, int verify, uint32_t *crc, uint32_t *hdr,
                         uint8_t *ok, uint32_t *nbad, uint32_t *pay = nullptr, bool route_cpu = true)
{
    if (!base && n) return fail(VAL_ERR_INVALID_ARG, "base is NULL");
    if ((off == nullptr) != (len == nullptr)) return fail(VAL_ERR_INVALID_ARG, "off/len must both be set or both NULL");
    const uint64_t tail = verify ? 4u : 0u;
    uint32_t lmin = UINT32_MAX, lmax = 0;
    uint64_t total = 0;
    bool monotone = true;
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t o = off ? off[i] : (uint64_t)i * stride;
        const uint64_t l = len ? len[i] : flen;
        if (o > base_len || l + tail > base_len - o) return fail(VAL_ERR_INVALID_ARG, "frame overruns the buffer");
        lmin = std::min<uint32_t>(lmin, (uint32_t)l);
        lmax = std::max<uint32_t>(lmax, (uint32_t)l);
        total += l;
        if (off && i && off[i] < off[i - 1]) monotone = false;
    }
    if (route_cpu && total < host_batch_min_bytes(n ? total / n : 0)) {  // below the crossover: the CPU engine
        const uint32_t bad = cpu_frames(base, off, len, stride, flen, n, total, verify, crc, hdr, ok, pay);
        if (nbad) *nbad = verify ? bad : 0u;
        return VAL_OK;
    }
    DeviceScope ds;
    Ctx *cp = nullptr;
    val_status_t st = cur(&cp);
    if (st != VAL_OK) return st;
    Ctx &c = *cp;
    std::lock_guard<std::recursive_mutex> lk(c.mu);
    const size_t desc_bytes = off ? (size_t)n * 12u : 0u;
    const size_t out_bytes = (size_t)n * 13u + 16u;
    if (n) {
        uint64_t lo = UINT64_MAX, hi = 0;
        for (uint32_t i = 0; i < n; i++) {
            const uint64_t o = off ? off[i] : (uint64_t)i * stride;
            lo = std::min(lo, o);
            hi = std::max(hi, o + (len ? len[i] : flen) + tail);
        }
        if (hi - lo <= kHostZeroCopy)
            return frames_host_small(c, base, lo, hi, off, len, stride, flen, n, verify, lmin == lmax ? lmax : 0u, crc,
                                     hdr, ok, nbad, pay);
    }
    if ((st = grow(&c.d_small, &c.d_small_cap, desc_bytes + out_bytes + 64)) != VAL_OK) return st;
    hipStream_t s = c.stream, cs = c.copy;
    uint8_t *sm = c.d_small;
    uint64_t *d_off = off ? reinterpret_cast<uint64_t *>(sm) : nullptr;
    uint32_t *d_len = off ? reinterpret_cast<uint32_t *>(sm + (size_t)n * 8u) : nullptr;
    uint32_t *d_crc = reinterpret_cast<uint32_t *>(sm + desc_bytes);
    uint32_t *d_hdr = d_crc + n;
    uint32_t *d_pay = d_hdr + n;
    uint32_t *d_nbad = d_pay + n;
    uint8_t *d_ok = reinterpret_cast<uint8_t *>(d_nbad + 4);
    if (off && (size_t)n * 12u <= host_chunk_bytes()) {
        // both descriptor arrays through one bounce and one H2D (d_len follows d_off)
        if ((st = grow_pinned(&c.h_bounce[0], &c.h_bounce_cap[0], (size_t)n * 12u)) != VAL_OK) return st;
        VCRC_HIP(hipEventSynchronize(c.h2d_done[0]), "hipEventSynchronize");
        memcpy(c.h_bounce[0], off, (size_t)n * 8u);
        memcpy(c.h_bounce[0] + (size_t)n * 8u, len, (size_t)n * 4u);
        VCRC_HIP(hipMemcpyAsync(d_off, c.h_bounce[0], (size_t)n * 12u, hipMemcpyHostToDevice, s), "H2D descriptors");
        VCRC_HIP(hipEventRecord(c.h2d_done[0], s), "hipEventRecord");
    } else if (off) {
        if ((st = h2d_staged(c, reinterpret_cast<uint8_t *>(d_off), reinterpret_cast<const uint8_t *>(off),
                             (size_t)n * 8u, s)) != VAL_OK)
            return st;
        if ((st = h2d_staged(c, reinterpret_cast<uint8_t *>(d_len), reinterpret_cast<const uint8_t *>(len),
                             (size_t)n * 4u, s)) != VAL_OK)
            return st;
    }
    VCRC_HIP(hipMemsetAsync(d_nbad, 0, 4, s), "memset");
    // chunks of whole frames [i0, i1) covering wire bytes [lo, hi)
    const size_t cap = host_chunk_bytes();
    struct Chunk {
        uint32_t i0, i1;
        uint64_t lo, hi;
    };
    std::vector<Chunk> chunks;
    auto o_of = [&](uint32_t i) { return off ? off[i] : (uint64_t)i * stride; };
    auto e_of = [&](uint32_t i) { return o_of(i) + (len ? len[i] : flen) + tail; };
    if (off && !monotone) {
        Chunk ch{0, n, UINT64_MAX, 0};
        for (uint32_t i = 0; i < n; i++) {
            ch.lo = std::min(ch.lo, o_of(i));
            ch.hi = std::max(ch.hi, e_of(i));
        }
        if (n) chunks.push_back(ch);
    } else {
        for (uint32_t i = 0; i < n;) {
            Chunk ch{i, i + 1, o_of(i), e_of(i)};
            while (ch.i1 < n && std::max(ch.hi, e_of(ch.i1)) - ch.lo <= cap) ch.hi = std::max(ch.hi, e_of(ch.i1++));
            chunks.push_back(ch);
            i = ch.i1;
        }
    }
    size_t slot_need = 1;
    for (const Chunk &ch : chunks) slot_need = std::max<size_t>(slot_need, (size_t)(ch.hi - ch.lo));
    const bool pinned = n && is_pinned(base);
    for (int k = 0; k < 2; k++) {
        if ((st = grow(&c.d_slot[k], &c.d_slot_cap[k], slot_need)) != VAL_OK) return st;
        if (!pinned && n && (st = grow_pinned(&c.h_bounce[k], &c.h_bounce_cap[k], slot_need)) != VAL_OK) return st;
    }
    // no slot may be refilled before the previous call's kernels finished with it
    VCRC_HIP(hipEventRecord(c.kern_done[0], s), "hipEventRecord");
    VCRC_HIP(hipEventRecord(c.kern_done[1], s), "hipEventRecord");
    const uint32_t hint = (off && lmin != lmax) ? 0u : lmax;
    for (size_t ci = 0; ci < chunks.size(); ci++) {
        const Chunk &ch = chunks[ci];
        const int k = (int)(ci & 1);
        const size_t bytes = (size_t)(ch.hi - ch.lo);
        VCRC_HIP(hipStreamWaitEvent(cs, c.kern_done[k], 0), "hipStreamWaitEvent");
        if (pinned) {
            VCRC_HIP(hipMemcpyAsync(c.d_slot[k], base + ch.lo, bytes, hipMemcpyHostToDevice, cs), "H2D frames");
        } else {
            VCRC_HIP(hipEventSynchronize(c.h2d_done[k]), "hipEventSynchronize");  // bounce k drained
            parallel_copy(c.h_bounce[k], base + ch.lo, bytes);
            VCRC_HIP(hipMemcpyAsync(c.d_slot[k], c.h_bounce[k], bytes, hipMemcpyHostToDevice, cs), "H2D frames");
        }
        VCRC_HIP(hipEventRecord(c.h2d_done[k], cs), "hipEventRecord");
        VCRC_HIP(hipStreamWaitEvent(s, c.h2d_done[k], 0), "hipStreamWaitEvent");
        FrameParams p{};
        p.base = c.d_slot[k] - ch.lo;  // the kernel only touches base + off within the slot
        p.off = d_off ? d_off + ch.i0 : nullptr;
        p.len = d_len ? d_len + ch.i0 : nullptr;
        if (!off) p.base = c.d_slot[k];  // strided: frame i0 is at the slot start
        p.stride = stride;
        p.flen = flen;
        p.last_len = flen;
        p.n = ch.i1 - ch.i0;
        p.seed0 = p.seed_rest = 0xFFFFFFFFu;
        p.xorout = 0xFFFFFFFFu;
        p.out_crc = crc ? d_crc + ch.i0 : nullptr;
        p.out_hdr = hdr ? d_hdr + ch.i0 : nullptr;
        p.verify = verify ? 1u : 0u;
        p.out_ok = ok ? d_ok + ch.i0 : nullptr;
        p.nbad = d_nbad;
        p.out_pay = pay ? d_pay + ch.i0 : nullptr;
        if ((st = launch_frames(c, p, hint, s)) != VAL_OK) return st;
        VCRC_HIP(hipEventRecord(c.kern_done[k], s), "hipEventRecord");
    }
    // results land in pinned memory (d_crc | d_hdr | d_pay | d_nbad | d_ok are contiguous), then are copied out
    if ((st = grow_pinned(&c.h_out, &c.h_out_cap, out_bytes)) != VAL_OK) return st;
    VCRC_HIP(hipMemcpyAsync(c.h_out, d_crc, out_bytes, hipMemcpyDeviceToHost, s), "D2H results");
    VCRC_HIP(hipStreamSynchronize(s), "hipStreamSynchronize");
    const uint8_t *h = c.h_out;
    if (crc) memcpy(crc, h, (size_t)n * 4u);
    if (hdr) memcpy(hdr, h + (size_t)n * 4u, (size_t)n * 4u);
    if (pay) memcpy(pay, h + (size_t)n * 8u, (size_t)n * 4u);
    uint32_t bad = 0;
    memcpy(&bad, h + (size_t)n * 12u, 4);
    if (ok) memcpy(ok, h + (size_t)n * 12u + 16u, (size_t)n);
    if (nbad) *nbad = bad;
    return VAL_OK;
}

// ---- several devices in one process -------------------------------
// Frames are independent: a batch is cut into ndev contiguous frame ranges
// balanced by CRC-input bytes; one host thread per range binds to device
// (range % device count) and runs the single-device host path on it, writing
// a disjoint range of the outputs. No collective, no peer traffic. Ranges
// that share a device serialise on its context.
// All world + 1 cuts in one pass: cut r = the first frame whose byte prefix
// sum reaches total * r / world (count-balanced when len is NULL).
std::vector<uint32_t> shard_cuts(uint32_t n, const uint32_t *len, uint32_t world)
{
    std::vector<uint32_t> cut(world + 1, n);
    cut[0] = 0;
    if (!len) {
        const uint32_t base = n / world, extra = n % world;
        for (uint32_t r = 1; r < world; r++) cut[r] = r * base + std::min(r, extra);
        return cut;
    }
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; i++) total += len[i];
    uint64_t acc = 0;
    uint32_t i = 0;
    for (uint32_t r = 1; r < world; r++) {
        const uint64_t target = (uint64_t)((__uint128_t)total * r / world);
        while (i < n && acc < target) acc += len[i++];
        cut[r] = i;
    }
    return cut;
}

void shard_frames(uint32_t n, const uint32_t *len, uint32_t world, uint32_t rank, uint32_t *start, uint32_t *count)
{
    const std::vector<uint32_t> cut = shard_cuts(n, len, world);
    *start = cut[rank];
    *count = cut[rank + 1] - cut[rank];
}

// CPU or GPU for a whole host batch over `devices` distinct GPUs (the
// *_host_multi calls decide once, never per shard). The single-GPU crossover
// C1 (host_batch_min_bytes) was measured against one CPU thread. With N
// devices each shard's H2D runs on its own PCIe link and DMA engines while
// the fixed costs (launch, completion wait, first chunk) are paid
// concurrently, so for pinned input the GPU side's byte rate scales with N;
// the CPU engine's scales with its T threads (val_gpu_set_host_cpu_threads,
// capped by the CPU budget): C(N, T) = C1 * T / N.
// Pageable input also passes through the host bounce copies, which all
// shards share inside the process's CPU budget. Measured on the GPU box
// (16 CPUs, tools/bounce_copy_scaling.py, profiles/r06_bounce_copy_scaling.
// jsonl): one copy thread moves about 14 GB/s and all copies together
// saturate near 135 GB/s (112 / 124 / 151 / 136 GB/s at 1 / 2 / 4 / 8
// concurrent 64 MiB copies), while one GPU's pageable host path takes about
// 53 GB/s. So N pageable shards feed at most N_eff = min(N, R_copy(N) / 53)
// devices' worth of GPU (2.55 at N >= 4 on the box), and C(N, T) = C1 * T /
// N_eff. A GPU test that forces C1 = 0 keeps every batch on the GPU.
#ifndef VCRC_COPY_MBS_PER_THREAD
#define VCRC_COPY_MBS_PER_THREAD 14000u  // MB/s one bounce-copy thread moves
#endif
#ifndef VCRC_COPY_MBS_MAX
#define VCRC_COPY_MBS_MAX 135000u  // MB/s all bounce copies of the process together
#endif
#ifndef VCRC_PAGEABLE_MBS_PER_GPU
#define VCRC_PAGEABLE_MBS_PER_GPU 53000u  // MB/s of one GPU's pageable host path (49.6 GiB/s)
#endif

// N_eff * 16 for `devices` shards (pinned: N * 16).
uint64_t host_multi_devices_x16(int devices, bool pinned)
{
    const uint64_t n = (uint64_t)std::max(1, devices);
    if (pinned) return n * 16u;
    const uint64_t threads =
        std::min<uint64_t>(host_cpu_budget(), n * copy_threads(host_chunk_bytes(), (uint32_t)n));
    const uint64_t copy = std::min<uint64_t>(threads * VCRC_COPY_MBS_PER_THREAD, VCRC_COPY_MBS_MAX);
    return std::max<uint64_t>(16u, std::min<uint64_t>(n * 16u, copy * 16u / VCRC_PAGEABLE_MBS_PER_GPU));
}

uint64_t host_multi_min_bytes(int devices, uint64_t mean_len = UINT64_MAX, bool pinned = false)
{
    const uint64_t t = std::max<uint64_t>(1, std::min<uint64_t>(g_host_cpu_threads.load(), host_cpu_budget()));
    return host_batch_min_bytes(mean_len) * t * 16u / host_multi_devices_x16(devices, pinned);
}

// Run work(0..k-1): k-1 helper threads plus the calling thread; a helper that
// cannot be started leaves its index to the calling thread.
template <typename F>
void run_shards(int k, F &&work)
{
    std::vector<std::thread> th;
    int started = 1;
    for (; started < k; started++) {
        try {
            th.emplace_back(work, started);
        } catch (...) {
            break;
        }
    }
    work(0);
    for (int d = started; d < k; d++) work(d);
    for (auto &x : th) x.join();
}

val_status_t frames_host_multi(const uint8_t *base, uint64_t base_len, const uint64_t *off, const uint32_t *len,
                               uint64_t stride, uint32_t flen, uint32_t n, int verify, uint32_t *crc, uint32_t *hdr,
                               uint8_t *ok, uint32_t *nbad, int ndev)
{
    if (!base && n) return fail(VAL_ERR_INVALID_ARG, "base is NULL");
    if ((off == nullptr) != (len == nullptr)) return fail(VAL_ERR_INVALID_ARG, "off/len must both be set or both NULL");
    const uint64_t tail = verify ? 4u : 0u;
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t o = off ? off[i] : (uint64_t)i * stride;
        const uint64_t l = len ? len[i] : flen;
        if (o > base_len || l + tail > base_len - o) return fail(VAL_ERR_INVALID_ARG, "frame overruns the buffer");
        total += l;
    }
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count < 0) {
        (void)hipGetLastError();
        count = 0;
    }
    if (ndev <= 0) ndev = std::max(1, std::min(count, kMaxDevices));
    ndev = std::min(ndev, kMaxDevices);
    // one decision for the whole batch: distinct devices the shards land on
    if (total < host_multi_min_bytes(std::max(1, std::min(ndev, count)), n ? total / n : 0,
                                 n && count > 0 && is_pinned(base))) {
        const uint32_t bad = cpu_frames(base, off, len, stride, flen, n, total, verify, crc, hdr, ok, nullptr);
        if (nbad) *nbad = verify ? bad : 0u;
        return VAL_OK;
    }
    if (count <= 0) return fail(VAL_ERR_IO, "no HIP device");
    std::vector<val_status_t> st(ndev, VAL_OK);
    std::vector<uint32_t> bad(ndev, 0);
    std::vector<std::string> err(ndev);
    const std::vector<uint32_t> cut = shard_cuts(n, len, (uint32_t)ndev);
    auto work = [&](int d) {
        const int prev = t_dev;
        t_dev = d % count;  // more shards than devices share them round-robin
        const uint32_t s0 = cut[d], cnt = cut[d + 1] - cut[d];
        const bool strided = off == nullptr;
        const uint8_t *b = strided ? base + (uint64_t)s0 * stride : base;
        const uint64_t bl = strided ? base_len - std::min<uint64_t>(base_len, (uint64_t)s0 * stride) : base_len;
        st[d] = frames_host(b, bl, strided ? nullptr : off + s0, strided ? nullptr : len + s0, stride, flen, cnt, verify,
                            crc ? crc + s0 : nullptr, hdr ? hdr + s0 : nullptr, ok ? ok + s0 : nullptr, &bad[d],
                            nullptr, /*route_cpu=*/false);
        err[d] = t_err;
        t_dev = prev;
    };
    run_shards(ndev, work);
    uint32_t total_bad = 0;
    for (int d = 0; d < ndev; d++) {
        if (st[d] != VAL_OK) {
            t_err = "device " + std::to_string(d) + ": " + err[d];
            return st[d];
        }
        total_bad += bad[d];
    }
    if (nbad) *nbad = total_bad;
    return VAL_OK;
}

// One long host window split into byte ranges, one per device (4 KiB
// aligned); device 0's range starts from state_in, the others from 0; the
// partial raw states fold in order with the GF(2) shift. Below the N-device
// crossover (host_multi_min_bytes, decided once for the whole window) the CPU
// engine folds the window on the calling thread plus helper threads (>= 4 MiB
// each, within the CPU budget), the same way.
val_status_t region_host_multi(const void *data, uint64_t len, uint32_t state_in, uint32_t *state_out, int ndev)
{
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count < 0) {
        (void)hipGetLastError();
        count = 0;
    }
    if (ndev <= 0) ndev = std::max(1, std::min(count, kMaxDevices));
    ndev = std::min(ndev, kMaxDevices);
    const bool on_cpu =
        len < host_multi_min_bytes(std::max(1, std::min(ndev, count)), UINT64_MAX, len && count > 0 && is_pinned(data));
    if (!on_cpu && count <= 0) return fail(VAL_ERR_IO, "no HIP device");
    int parts = ndev;
    if (on_cpu) {
        g_cpu_batches.fetch_add(1, std::memory_order_relaxed);
        parts = (int)std::max<uint64_t>(1, std::min<uint64_t>({(uint64_t)g_host_cpu_threads.load(),
                                                               (uint64_t)host_cpu_budget(), len >> 22}));
    }
    const uint64_t per = ((len + parts - 1) / parts + 4095u) & ~(uint64_t)4095u;
    std::vector<val_status_t> st(parts, VAL_OK);
    std::vector<uint32_t> part(parts, 0);
    std::vector<uint64_t> plen(parts, 0);
    std::vector<std::string> err(parts);
    auto work = [&](int d) {
        const uint64_t lo = std::min(len, (uint64_t)d * per), hi = std::min(len, lo + per);
        const uint8_t *p = static_cast<const uint8_t *>(data) + lo;
        plen[d] = hi - lo;
        if (on_cpu) {
            part[d] = vcrc_cpu_update(d == 0 ? state_in : 0u, p, (size_t)(hi - lo));
            return;
        }
        const int prev = t_dev;
        t_dev = d % count;  // more shards than devices share them round-robin
        st[d] = region_host(p, (size_t)(hi - lo), d == 0 ? state_in : 0u, &part[d]);
        err[d] = t_err;
        t_dev = prev;
    };
    run_shards(parts, work);
    uint32_t acc = 0;
    for (int d = 0; d < parts; d++) {
        if (st[d] != VAL_OK) {
            t_err = "device " + std::to_string(d) + ": " + err[d];
            return st[d];
        }
        acc = (d == 0 ? part[0] : gf2_mul(gf2_x8n(plen[d]), acc) ^ part[d]);
    }
    *state_out = acc;
    return VAL_OK;
}

// Rolling file CRC of the RX path from the payload states (reference
// src/val_receiver.c:794,891: crc_state = val_crc32_update_state(crc_state,
// payload) per in-order frame): state = shift(state, pay_len) ^ pay_state,
// frame after frame. x^(8 pay_len) is cached as a nibble map per distinct
// length, so a window of equal frames costs 8 lookups per frame.
struct ShiftMap {
    uint64_t n = UINT64_MAX;
    uint32_t t[8][16];
    void set(uint64_t bytes)
    {
        if (bytes == n) return;
        const uint32_t x = gf2_x8n(bytes);
        for (int k = 0; k < 8; k++)
            for (int v = 0; v < 16; v++) t[k][v] = gf2_mul(x, (uint32_t)v << (4 * k));
        n = bytes;
    }
    uint32_t apply(uint32_t a) const
    {
        uint32_t r = 0;
        for (int k = 0; k < 8; k++) r ^= t[k][(a >> (4 * k)) & 15u];
        return r;
    }
};

uint32_t fold_payloads(uint32_t state, const uint32_t *pay_state, const uint32_t *pay_len, const uint8_t *ok,
                       uint32_t n, uint32_t *n_folded)
{
    ShiftMap m;
    uint32_t i = 0;
    for (; i < n && (!ok || ok[i]); i++) {
        m.set(pay_len[i]);
        state = m.apply(state) ^ pay_state[i];
    }
    if (n_folded) *n_folded = i;
    return state;
}

// The same fold with the receiver's ordering rule (reference
// src/val_receiver.c:871-891, offsets from src/val_core.c:981-993): a DATA
// frame whose effective offset (its explicit offset, or *written when the
// offset is implied) equals *written is folded and advances *written by its
// payload; an earlier offset is a duplicate and a later one a gap: neither
// is folded, and later frames are still judged one by one, as the receiver
// does. Frames with ok[i] == 0 (trailer mismatch) and non-DATA frames
// (VAL_FRAME_OFFSET_NOT_DATA) are never folded.
uint32_t fold_payloads_at(uint32_t state, const uint32_t *pay_state, const uint32_t *pay_len, const uint64_t *file_off,
                          const uint8_t *ok, uint32_t n, uint64_t *written, uint32_t *n_folded)
{
    ShiftMap m;
    uint64_t w = *written;
    uint32_t folded = 0;
    for (uint32_t i = 0; i < n; i++) {
        if ((ok && !ok[i]) || file_off[i] == VAL_FRAME_OFFSET_NOT_DATA) continue;
        const uint64_t eff = file_off[i] == VAL_FRAME_OFFSET_IMPLIED ? w : file_off[i];
        if (eff != w) continue;
        m.set(pay_len[i]);
        state = m.apply(state) ^ pay_state[i];
        w += pay_len[i];
        folded++;
    }
    *written = w;
    if (n_folded) *n_folded = folded;
    return state;
}

void ctx_free(Ctx &c)
{
    if (c.device >= 0) (void)hipSetDevice(c.device);
    if (c.stream) (void)hipStreamSynchronize(c.stream);
    if (c.copy) (void)hipStreamSynchronize(c.copy);
    if (c.d_stage) (void)hipFree(c.d_stage);
    if (c.d_small) (void)hipFree(c.d_small);
    if (c.d_consts) (void)hipFree(c.d_consts);
    for (int k = 0; k < 2; k++) {
        if (c.d_slot[k]) (void)hipFree(c.d_slot[k]);
        if (c.h_bounce[k]) (void)hipHostFree(c.h_bounce[k]);
        if (c.h2d_done[k]) (void)hipEventDestroy(c.h2d_done[k]);
        if (c.kern_done[k]) (void)hipEventDestroy(c.kern_done[k]);
    }
    (void)hipDeviceSynchronize();  // the streams that used the scratch may be gone
    for (StreamScratch *x : c.scratch) scratch_free(x);
    c.scratch.clear();
    if (c.h_out) (void)hipHostFree(c.h_out);
    if (c.copy) (void)hipStreamDestroy(c.copy);
    if (c.stream) (void)hipStreamDestroy(c.stream);
}

}  // namespace vcrc

using namespace vcrc;

extern "C" {

val_status_t val_gpu_init(int device)
{
    t_err.clear();
    if (device < 0) device = 0;
    Ctx *c = nullptr;
    val_status_t st = get_ctx(device, &c);
    if (st != VAL_OK) return st;
    t_dev = device;
    VCRC_HIP(hipSetDevice(device), "hipSetDevice");
    return VAL_OK;
}

int val_gpu_init_devices(int n)
{
    t_err.clear();
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        fail(VAL_ERR_IO, "val_gpu_init_devices: no HIP device");
        return 0;
    }
    if (n <= 0 || n > count) n = std::min(count, kMaxDevices);
    for (int d = 0; d < n; d++) {
        Ctx *c = nullptr;
        if (get_ctx(d, &c) != VAL_OK) return d;
    }
    return n;
}

val_status_t val_gpu_set_device(int device)
{
    t_err.clear();
    Ctx *c = nullptr;
    val_status_t st = get_ctx(device, &c);
    if (st != VAL_OK) return st;
    t_dev = device;
    VCRC_HIP(hipSetDevice(device), "hipSetDevice");
    return VAL_OK;
}

int val_gpu_current_device(void)
{
    const int d = t_dev >= 0 ? t_dev : g_default_dev.load(std::memory_order_relaxed);
    return d;
}

void val_gpu_shutdown(void)
{
    std::lock_guard<std::mutex> lk(g_ctx_mu);
    for (int d = 0; d < kMaxDevices; d++) {
        Ctx *c = g_ctxs[d].exchange(nullptr);
        if (!c) continue;
        {
            std::lock_guard<std::recursive_mutex> lk2(c->mu);
            ctx_free(*c);
        }
        delete c;
    }
    g_default_dev.store(-1);
    t_dev = -1;
}

int val_gpu_device_count(void)
{
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess) return 0;
    return c;
}

uint32_t val_gpu_abi_version(void) { return VAL_GPU_ABI_VERSION; }

#ifdef VCRC_TIMING
// Diagnostic builds only: copy the per-wave stamps of the last k_frames launch.
int vcrc_debug_times(uint64_t *out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vcrc_time), sizeof(g_vcrc_time)) == hipSuccess ? 0 : -1;
}
int vcrc_debug_info(uint32_t *out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_vcrc_info), sizeof(g_vcrc_info)) == hipSuccess ? 0 : -1;
}
#endif

const char *val_gpu_last_error(void) { return t_err.c_str(); }

const char *val_gpu_build_flags(void)
{
    // every compile-time switch of the sources, diagnostic or A/B, that is set
    static const char flags[] = ""
#ifdef VCRC_DIAG_BUILD
                                " VCRC_DIAG_BUILD"
#endif
#ifdef VCRC_DIAG_NOHASH
                                " VCRC_DIAG_NOHASH"
#endif
#ifdef VCRC_NO_LDS_FILL
                                " VCRC_NO_LDS_FILL"
#endif
#ifdef VCRC_REGION_HASHONLY
                                " VCRC_REGION_HASHONLY"
#endif
#ifdef VCRC_REGION_NOATOMIC
                                " VCRC_REGION_NOATOMIC"
#endif
#ifdef VCRC_TIMING
                                " VCRC_TIMING"
#endif
#ifdef VCRC_NO_SPLIT
                                " VCRC_NO_SPLIT"
#endif
#ifdef VCRC_NO_KARG_EARLY
                                " VCRC_NO_KARG_EARLY"
#endif
        ;
    return flags[0] ? flags + 1 : flags;
}

void val_gpu_set_provider_min_bytes(int64_t bytes) { g_provider_min.store(bytes < 0 ? -1 : bytes); }

uint64_t val_gpu_provider_min_bytes(void) { return provider_min_bytes(); }

void val_gpu_set_host_batch_min_bytes(int64_t bytes) { g_host_batch_min.store(bytes < 0 ? -1 : bytes); }

uint64_t val_gpu_host_batch_min_bytes(void) { return host_batch_min_bytes(); }

uint64_t val_gpu_host_batch_min_bytes_for(uint64_t mean_len) { return host_batch_min_bytes(mean_len); }

uint64_t val_gpu_cpu_batch_count(void) { return g_cpu_batches.load(std::memory_order_relaxed); }

void val_gpu_set_host_cpu_threads(uint32_t threads)
{
    g_host_cpu_threads.store(std::max<uint32_t>(1, std::min<uint32_t>(threads, 256)));
}

uint64_t val_gpu_host_multi_min_bytes(int devices) { return host_multi_min_bytes(devices); }

void val_gpu_set_tail_pieces(int enable) { g_tail_pieces.store(enable < 0 ? -1 : (enable ? 1 : 0)); }

uint64_t val_gpu_tail_piece_launches(void) { return g_tail_piece_launches.load(std::memory_order_relaxed); }

uint64_t val_gpu_host_multi_min_bytes_ex(int devices, int pinned, uint64_t mean_len)
{
    return host_multi_min_bytes(devices, mean_len, pinned != 0);
}

void val_gpu_set_ragged_min_frames(int64_t frames) { g_ragged_min.store(frames < 0 ? -1 : frames); }

uint32_t val_gpu_ragged_min_frames(void) { return ragged_min_frames(); }

uint32_t val_gpu_scratch_entries(int device, uint64_t *evictions)
{
    if (evictions) *evictions = 0;
    if (device < 0 || device >= kMaxDevices) return 0;
    Ctx *c = g_ctxs[device].load(std::memory_order_acquire);
    if (!c) return 0;
    std::lock_guard<std::recursive_mutex> lk(c->mu);
    if (evictions) *evictions = c->scratch_evictions;
    return (uint32_t)c->scratch.size();
}

uint64_t val_gpu_cpu_small_count(void) { return cpu_small_total(); }

int val_gpu_last_hook_path(void) { return t_hook_path; }

uint32_t val_crc32_cpu_update_state(uint32_t state, const void *data, size_t len, int engine)
{
    if (len && !data) return state;
    return vcrc_cpu_update_with(engine, state, data, len);
}

int val_crc32_cpu_engine(void) { return vcrc_cpu_engine(); }

uint32_t val_gpu_host_copy_threads(uint64_t bytes, uint32_t concurrent_copies)
{
    return copy_threads(bytes, concurrent_copies);
}

val_status_t val_gpu_host_copy_probe(uint32_t copies, uint64_t bytes, uint32_t reps, int pinned_dst, double *gbs)
{
    if (!copies || copies > 64 || !bytes || !reps || !gbs) return fail(VAL_ERR_INVALID_ARG, "copy probe arguments");
    *gbs = 0.0;
    std::vector<uint8_t *> src(copies, nullptr), dst(copies, nullptr);
    val_status_t st = VAL_OK;
    for (uint32_t i = 0; i < copies && st == VAL_OK; i++) {
        src[i] = static_cast<uint8_t *>(malloc(bytes));
        if (!src[i]) {
            st = fail(VAL_ERR_NO_MEMORY, "copy probe: source");
            break;
        }
        memset(src[i], (int)(i + 1), bytes);  // resident, like a transport's window
        if (pinned_dst) {
            const hipError_t e = hipHostMalloc((void **)&dst[i], bytes, hipHostMallocDefault);
            if (e != hipSuccess) {
                dst[i] = nullptr;
                st = fail(VAL_ERR_IO, "copy probe: hipHostMalloc", e);
            }
        } else if (!(dst[i] = static_cast<uint8_t *>(malloc(bytes)))) {
            st = fail(VAL_ERR_NO_MEMORY, "copy probe: destination");
        }
        if (dst[i]) memset(dst[i], 0, bytes);
    }
    if (st == VAL_OK) {
        // every copy stream starts together; the span is first start to last end
        std::atomic<uint32_t> ready{0};
        std::atomic<bool> go{false};
        auto work = [&](int i) {
            ready.fetch_add(1);
            while (!go.load(std::memory_order_acquire)) std::this_thread::yield();
            for (uint32_t r = 0; r < reps; r++) parallel_copy(dst[i], src[i], bytes);
        };
        std::vector<std::thread> th;
        try {
            for (uint32_t i = 1; i < copies; i++) th.emplace_back(work, (int)i);
        } catch (...) {
            st = fail(VAL_ERR_NO_MEMORY, "copy probe: thread");
        }
        while (ready.load() < (uint32_t)th.size()) std::this_thread::yield();
        const auto t0 = std::chrono::steady_clock::now();
        go.store(true, std::memory_order_release);
        if (st == VAL_OK) work(0);
        for (auto &x : th) x.join();
        const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (st == VAL_OK) *gbs = (double)bytes * reps * copies / s / 1e9;
    }
    for (uint32_t i = 0; i < copies; i++) {
        free(src[i]);
        if (dst[i]) {
            if (pinned_dst) (void)hipHostFree(dst[i]);
            else free(dst[i]);
        }
    }
    return st;
}

uint64_t val_gpu_cpu_fallback_count(void) { return g_cpu_fallbacks.load(std::memory_order_relaxed); }

void val_gpu_set_cpu_fallback(int enable) { g_cpu_fallback_on.store(enable < 0 ? -1 : (enable ? 1 : 0)); }

uint32_t val_gpu_lanes_per_frame(uint32_t typical_len) { return lanes_per_frame(typical_len); }

val_status_t val_gpu_set_lanes_per_frame(uint32_t lanes)
{
    if (lanes != 0 && !valid_lanes(lanes)) return fail(VAL_ERR_INVALID_ARG, "lanes must be 0 or a power of two <= 64");
    g_forced_lanes.store(lanes, std::memory_order_relaxed);
    return VAL_OK;
}

val_status_t val_gpu_set_host_chunk_bytes(size_t bytes)
{
    g_host_chunk.store(bytes, std::memory_order_relaxed);
    return VAL_OK;
}

void *val_gpu_host_alloc(size_t bytes)
{
    DeviceScope ds;
    Ctx *c = nullptr;
    if (cur(&c) != VAL_OK) return nullptr;
    void *p = nullptr;
    hipError_t e = hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault);
    if (e != hipSuccess) {
        fail(VAL_ERR_NO_MEMORY, "hipHostMalloc", e);
        return nullptr;
    }
    return p;
}

void val_gpu_host_free(void *p)
{
    if (p) (void)hipHostFree(p);
}

val_status_t val_gpu_set_prefetch(int depth)
{
    if (depth != -1 && !valid_prefetch(depth))
        return fail(VAL_ERR_INVALID_ARG, "prefetch depth must be -1, 0, 1, 2, 4, -2 or -3");
    g_forced_prefetch.store(depth, std::memory_order_relaxed);
    return VAL_OK;
}

uint32_t val_crc32_shift(uint32_t state, uint64_t nbytes) { return gf2_mul(gf2_x8n(nbytes), state); }

uint32_t val_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b)
{
    return gf2_mul(gf2_x8n(len_b), crc_a) ^ crc_b;
}

uint32_t val_crc32_fold_partials(const uint32_t *state, const uint64_t *nbytes, uint32_t k)
{
    uint32_t acc = 0;
    for (uint32_t i = 0; i < k; i++) acc = (i == 0 ? state[0] : gf2_mul(gf2_x8n(nbytes[i]), acc) ^ state[i]);
    return acc;
}

void val_shard_frames(uint32_t n, const uint32_t *len, uint32_t world, uint32_t rank, uint32_t *start, uint32_t *count)
{
    if (!start || !count) return;
    if (world == 0 || rank >= world) {
        *start = *count = 0;
        return;
    }
    shard_frames(n, len, world, rank, start, count);
}

uint32_t val_crc32_init_state(void) { return 0xFFFFFFFFu; }

uint32_t val_crc32_finalize_state(uint32_t state) { return state ^ 0xFFFFFFFFu; }

uint32_t val_crc32_update_state(uint32_t state, const void *data, size_t length)
{
    return scalar_state("val_crc32_update_state", state, data, length);
}

uint32_t val_crc32(const void *data, size_t length)
{
    return scalar_state("val_crc32", 0xFFFFFFFFu, data, length) ^ 0xFFFFFFFFu;
}

uint32_t val_gpu_crc32_provider(uint32_t seed, const void *buf, size_t len)
{
    return scalar_state("val_gpu_crc32_provider", seed, buf, len) ^ 0xFFFFFFFFu;
}

val_status_t val_crc32_frames_dev(const uint8_t *d_base, const uint64_t *d_off, const uint32_t *d_len, uint64_t stride,
                                  uint32_t flen, uint32_t n, uint32_t len_hint, uint32_t *d_crc, uint32_t *d_hdr,
                                  void *stream)
{
    t_err.clear();
    if ((d_off == nullptr) != (d_len == nullptr)) return fail(VAL_ERR_INVALID_ARG, "off/len must both be set or both NULL");
    if (!d_base && n) return fail(VAL_ERR_INVALID_ARG, "base is NULL");
    DeviceScope ds;
    Ctx *c = nullptr;
    val_status_t st = cur_dev(stream, d_base, &c);
    if (st != VAL_OK) return st;
    FrameParams p{};
    p.base = d_base;
    p.off = d_off;
    p.len = d_len;
    p.stride = stride;
    p.flen = flen;
    p.last_len = flen;
    p.n = n;
    p.seed0 = p.seed_rest = 0xFFFFFFFFu;
    p.xorout = 0xFFFFFFFFu;
    p.out_crc = d_crc;
    p.out_hdr = d_hdr;
    return launch_frames(*c, p, d_off ? len_hint : flen, pick_stream(stream));
}

val_status_t val_crc32_verify_frames_dev(const uint8_t *d_base, const uint64_t *d_off, const uint32_t *d_len,
                                         uint64_t stride, uint32_t flen, uint32_t n, uint32_t len_hint, uint8_t *d_ok,
                                         uint32_t *d_nbad, uint32_t *d_crc, uint32_t *d_hdr, void *stream)
{
    t_err.clear();
    if ((d_off == nullptr) != (d_len == nullptr)) return fail(VAL_ERR_INVALID_ARG, "off/len must both be set or both NULL");
    if (!d_base && n) return fail(VAL_ERR_INVALID_ARG, "base is NULL");
    DeviceScope ds;
    Ctx *c = nullptr;
    val_status_t st = cur_dev(stream, d_base, &c);
    if (st != VAL_OK) return st;
    FrameParams p{};
    p.base = d_base;
    p.off = d_off;
    p.len = d_len;
    p.stride = stride;
    p.flen = flen;
    p.last_len = flen;
    p.n = n;
    p.seed0 = p.seed_rest = 0xFFFFFFFFu;
    p.xorout = 0xFFFFFFFFu;
    p.out_crc = d_crc;
    p.out_hdr = d_hdr;
    p.verify = 1;
    p.out_ok = d_ok;
    p.nbad = d_nbad;
    return launch_frames(*c, p, d_off ? len_hint : flen, pick_stream(stream));
}

val_status_t val_crc32_region_dev(const uint8_t *d_ptr, uint64_t len, uint32_t state_in, uint32_t *d_state_out,
                                  void *stream)
{
    t_err.clear();
    if (!d_state_out || (!d_ptr && len)) return fail(VAL_ERR_INVALID_ARG, "NULL pointer");
    DeviceScope ds;
    Ctx *c = nullptr;
    val_status_t st = cur_dev(stream, d_ptr, &c);
    if (st != VAL_OK) return st;
    return region_dev(*c, d_ptr, len, state_in, d_state_out, pick_stream(stream));
}

uint64_t val_crc32_region_scratch_bytes(uint64_t len) { return len > kRegionOneFrame ? 128u : 0u; }

val_status_t val_crc32_frames_host(const uint8_t *base, uint64_t base_len, const uint64_t *off, const uint32_t *len,
                                   uint64_t stride, uint32_t flen, uint32_t n, uint32_t *crc, uint32_t *hdr)
{
    t_err.clear();
    return frames_host(base, base_len, off, len, stride, flen, n, 0, crc, hdr, nullptr, nullptr);
}

val_status_t val_crc32_verify_frames_host(const uint8_t *base, uint64_t base_len, const uint64_t *off,
                                          const uint32_t *len, uint64_t stride, uint32_t flen, uint32_t n, uint8_t *ok,
                                          uint32_t *nbad)
{
    t_err.clear();
    uint32_t bad = 0;
    val_status_t st = frames_host(base, base_len, off, len, stride, flen, n, 1, nullptr, nullptr, ok, &bad);
    if (nbad) *nbad = bad;
    if (st == VAL_OK && bad) return VAL_ERR_CRC;
    return st;
}

val_status_t val_crc32_frames_host_multi(const uint8_t *base, uint64_t base_len, const uint64_t *off,
                                         const uint32_t *len, uint64_t stride, uint32_t flen, uint32_t n, uint32_t *crc,
                                         uint32_t *hdr, int ndev)
{
    t_err.clear();
    return frames_host_multi(base, base_len, off, len, stride, flen, n, 0, crc, hdr, nullptr, nullptr, ndev);
}

val_status_t val_crc32_verify_frames_host_multi(const uint8_t *base, uint64_t base_len, const uint64_t *off,
                                                const uint32_t *len, uint64_t stride, uint32_t flen, uint32_t n,
                                                uint8_t *ok, uint32_t *nbad, int ndev)
{
    t_err.clear();
    uint32_t bad = 0;
    val_status_t st = frames_host_multi(base, base_len, off, len, stride, flen, n, 1, nullptr, nullptr, ok, &bad, ndev);
    if (nbad) *nbad = bad;
    if (st == VAL_OK && bad) return VAL_ERR_CRC;
    return st;
}

val_status_t val_crc32_verify_frames_ex_dev(const uint8_t *d_base, const uint64_t *d_off, const uint32_t *d_len,
                                            uint64_t stride, uint32_t flen, uint32_t n, uint32_t len_hint,
                                            uint8_t *d_ok, uint32_t *d_nbad, uint32_t *d_crc, uint32_t *d_hdr,
                                            uint32_t *d_pay, void *stream)
{
    t_err.clear();
    if ((d_off == nullptr) != (d_len == nullptr)) return fail(VAL_ERR_INVALID_ARG, "off/len must both be set or both NULL");
    if (!d_base && n) return fail(VAL_ERR_INVALID_ARG, "base is NULL");
    DeviceScope ds;
    Ctx *c = nullptr;
    val_status_t st = cur_dev(stream, d_base, &c);
    if (st != VAL_OK) return st;
    FrameParams p{};
    p.base = d_base;
    p.off = d_off;
    p.len = d_len;
    p.stride = stride;
    p.flen = flen;
    p.last_len = flen;
    p.n = n;
    p.seed0 = p.seed_rest = 0xFFFFFFFFu;
    p.xorout = 0xFFFFFFFFu;
    p.out_crc = d_crc;
    p.out_hdr = d_hdr;
    p.verify = 1;
    p.out_ok = d_ok;
    p.nbad = d_nbad;
    p.out_pay = d_pay;
    return launch_frames(*c, p, d_off ? len_hint : flen, pick_stream(stream));
}

val_status_t val_crc32_verify_frames_ex_host(const uint8_t *base, uint64_t base_len, const uint64_t *off,
                                             const uint32_t *len, uint64_t stride, uint32_t flen, uint32_t n,
                                             uint8_t *ok, uint32_t *nbad, uint32_t *pay)
{
    t_err.clear();
    uint32_t bad = 0;
    val_status_t st = frames_host(base, base_len, off, len, stride, flen, n, 1, nullptr, nullptr, ok, &bad, pay);
    if (nbad) *nbad = bad;
    if (st == VAL_OK && bad) return VAL_ERR_CRC;
    return st;
}

uint32_t val_crc32_fold_payload_states(uint32_t state, const uint32_t *pay_state, const uint32_t *pay_len,
                                       const uint8_t *ok, uint32_t n, uint32_t *n_folded)
{
    if (!pay_state || !pay_len) {
        if (n_folded) *n_folded = 0;
        return state;
    }
    return fold_payloads(state, pay_state, pay_len, ok, n, n_folded);
}

uint32_t val_crc32_fold_payload_states_at(uint32_t state, const uint32_t *pay_state, const uint32_t *pay_len,
                                          const uint64_t *file_off, const uint8_t *ok, uint32_t n, uint64_t *written,
                                          uint32_t *n_folded)
{
    if (!pay_state || !pay_len || !file_off || !written) {
        if (n_folded) *n_folded = 0;
        return state;
    }
    return fold_payloads_at(state, pay_state, pay_len, file_off, ok, n, written, n_folded);
}

val_status_t val_crc32_region_host_multi(const void *data, uint64_t len, uint32_t state_in, uint32_t *state_out,
                                         int ndev)
{
    t_err.clear();
    if (!state_out || (!data && len)) return fail(VAL_ERR_INVALID_ARG, "NULL pointer");
    return region_host_multi(data, len, state_in, state_out, ndev);
}

}  // extern "C"
