/*
 * val_crc32_gpu.h -- C ABI of the MI355X (gfx950) CRC-32 integrity path.
 * Exported by val_protocol_amd/libval_crc_hip.so. Plain C types only; HIP
 * streams travel as `void *` (a hipStream_t; NULL = the HIP default stream).
 *
 * What each entry point replaces in the reference (VAL v0.7):
 *   val_gpu_crc32_provider  -> a crc32_func_t for val_config_t.crc32_provider
 *                              (include/val_protocol.h:163-166, :264-266),
 *                              consumed by val_internal_crc32
 *                              (src/val_core.c:399-406) and the region CRC
 *                              (src/val_core.c:431-438)
 *   val_crc32, val_crc32_{init,update,finalize}_state
 *                           -> src/val_core.c:150-183 (declared in
 *                              val_protocol.h)
 *   val_crc32_frames_*      -> the per-frame trailer CRC of the TX path
 *                              (src/val_core.c:828-834), batched over a window
 *                              (src/val_sender.c:822-841); optional header_crc
 *   val_crc32_verify_frames_* -> the RX trailer check (src/val_core.c:963-974),
 *                              batched; counts mismatches like crc_errors++
 *   val_crc32_region_dev    -> val_internal_crc32_region (src/val_core.c:414-455)
 *                              for resume tail-verify windows up to and beyond
 *                              256 MiB (src/val_receiver.c:158-181)
 *   val_crc32_combine/shift -> GF(2) algebra used to split long windows and
 *                              shard batches across GPUs (no reference
 *                              counterpart; zlib's crc32_combine identity)
 *
 *   val_crc32_*_multi       -> the same batches split over several GPUs of
 *                              one process, one host thread per device
 *                              (a window of src/val_sender.c:
 *                              822-841 sharded by contiguous frame ranges)
 *
 * Batch, region and device calls compute on the GPU only and return
 * VAL_ERR_IO on a missing device or a HIP failure. The three scalar hooks
 * (provider, val_crc32, val_crc32_update_state) take host memory, have no
 * error channel and are called by VAL under its session mutex on every
 * frame: inputs below the provider threshold (val_gpu_provider_min_bytes)
 * are answered by this library's own CPU engine, where a GPU round trip
 * cannot win, so the drop-in is never slower than the reference's byte loop;
 * longer inputs run on the GPU. On a GPU failure the hooks return the CRC
 * from the same CPU engine and count it (val_gpu_cpu_fallback_count);
 * VAL_GPU_CPU_FALLBACK=0 or val_gpu_set_cpu_fallback(0) makes them abort.
 */
#ifndef VAL_CRC32_GPU_H
#define VAL_CRC32_GPU_H

#include <stddef.h>
#include <stdint.h>

#include "val_errors.h"

#ifdef __cplusplus
extern "C" {
#endif

#define VAL_GPU_ABI_VERSION 1u

/* ---- lifetime ---------------------------------------------------------- */
/* Initialise HIP device `device` (0-based) and bind the calling thread to it.
 * The first device initialised is the process default, used by threads that
 * never bound one; the first CRC call initialises device 0 if none was.
 * Each device has its own streams, constant tables, staging and scratch. */
val_status_t val_gpu_init(int device);
/* Initialise devices 0..n-1 (n <= 0: all). Returns how many are usable. */
int val_gpu_init_devices(int n);
/* Bind the calling thread to `device` (initialised on first use); later calls
 * of this thread run there. hipSetDevice is per thread in HIP. */
val_status_t val_gpu_set_device(int device);
/* Device the calling thread's calls run on (-1: none initialised yet). */
int val_gpu_current_device(void);
/* Release every device context of the process (not concurrently with other
 * calls of this library; contexts are re-created on the next call). */
void val_gpu_shutdown(void);
int val_gpu_device_count(void);
uint32_t val_gpu_abi_version(void);
/* Last HIP/validation error text of the calling thread ("" if none). */
const char *val_gpu_last_error(void);
/* Scalar-hook calls answered by the CPU because the GPU path failed. */
uint64_t val_gpu_cpu_fallback_count(void);
/* 1: failed scalar hooks use the CPU (default), 0: they abort, -1: from
 * VAL_GPU_CPU_FALLBACK (unset or non-"0" = on). */
void val_gpu_set_cpu_fallback(int enable);

/* ---- scalar hooks (host memory) --------------------------------------- */
uint32_t val_gpu_crc32_provider(uint32_t seed, const void *buf, size_t len);
/* Inputs shorter than this many bytes are answered on the CPU by the scalar
 * hooks (the measured crossover). Set with
 * val_gpu_set_provider_min_bytes (-1 = VAL_GPU_PROVIDER_MIN_BYTES from the
 * environment, else the built-in default; 0 = always the GPU). */
void val_gpu_set_provider_min_bytes(int64_t bytes);
uint64_t val_gpu_provider_min_bytes(void);
/* Scalar-hook calls answered on the CPU because they were below the threshold. */
uint64_t val_gpu_cpu_small_count(void);
/* Where the calling thread's last scalar-hook call was answered. */
#define VAL_GPU_HOOK_NONE 0     /* no call yet on this thread */
#define VAL_GPU_HOOK_GPU 1      /* on the GPU */
#define VAL_GPU_HOOK_CPU 2      /* on the CPU, below the threshold */
#define VAL_GPU_HOOK_FALLBACK 3 /* on the CPU after the GPU path failed */
int val_gpu_last_hook_path(void);
/* The library's CPU engine itself: raw register after feeding data[0, len)
 * to state (val_crc32_update_state semantics). engine: 0 = the best this CPU
 * has, 1 = slice-by-16, 2 = carry-less multiply (PCLMULQDQ), 3 = 512-bit
 * carry-less multiply (VPCLMULQDQ + AVX-512); an engine the CPU lacks runs
 * the next simpler one. val_crc32_cpu_engine() = the engine 0 selects. */
uint32_t val_crc32_cpu_update_state(uint32_t state, const void *data, size_t len, int engine);
int val_crc32_cpu_engine(void);
uint32_t val_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);
/* state * x^(8*nbytes) mod P: advance a raw register over nbytes zero bytes. */
uint32_t val_crc32_shift(uint32_t state, uint64_t nbytes);

/* ---- batch frames, device-resident (async on `stream`) ------------------
 * Frame i is the CRC input base[off_i, off_i + len_i):
 *   descriptor mode: d_off[i], d_len[i] (device arrays; stride/flen ignored)
 *   strided mode   : d_off == d_len == NULL, off_i = i*stride, len_i = flen
 * Outputs (device, n entries, any may be NULL):
 *   d_crc[i] = CRC-32 of frame i (the trailer value)
 *   d_hdr[i] = header_crc = CRC-32 of the first min(8, len_i) bytes
 * len_hint (descriptor mode): typical frame length when the batch is
 * uniform (picks the lanes-per-frame geometry directly); 0 = lengths mixed or
 * unknown: frames are binned by length class on the device and each class
 * runs its own geometry (ragged path, no host synchronisation).
 * Lengths may be 0 .. 2^32-1.                                          */
val_status_t val_crc32_frames_dev(const uint8_t *d_base, const uint64_t *d_off, const uint32_t *d_len, uint64_t stride,
                                  uint32_t flen, uint32_t n, uint32_t len_hint, uint32_t *d_crc, uint32_t *d_hdr,
                                  void *stream);

/* RX verify: frame i's stored trailer is the LE32 at base + off_i + len_i.
 * d_ok[i] = 1 if it equals the recomputed CRC else 0 (nullable);
 * *d_nbad (device u32, nullable) is INCREMENTED by the number of mismatches
 * (zero it first; mirrors metrics.crc_errors++). d_crc/d_hdr as above. */
val_status_t val_crc32_verify_frames_dev(const uint8_t *d_base, const uint64_t *d_off, const uint32_t *d_len,
                                         uint64_t stride, uint32_t flen, uint32_t n, uint32_t len_hint, uint8_t *d_ok,
                                         uint32_t *d_nbad, uint32_t *d_crc, uint32_t *d_hdr, void *stream);

/* RX verify plus the receiver's rolling file-CRC input as a by-product
 * (reference src/val_receiver.c:794,891,1004-1005, where
 * every in-order DATA payload goes through val_crc32_update_state): as
 * val_crc32_verify_frames_dev, and d_pay[i] (nullable) = the raw register
 * after feeding frame i's payload to a ZERO register. The payload is the CRC
 * input after the 8-byte header and, when flags (byte 1) has
 * VAL_DATA_OFFSET_PRESENT, the 8-byte offset (0 if the frame is shorter).
 * Fold the states into the file CRC with val_crc32_fold_payload_states. */
val_status_t val_crc32_verify_frames_ex_dev(const uint8_t *d_base, const uint64_t *d_off, const uint32_t *d_len,
                                            uint64_t stride, uint32_t flen, uint32_t n, uint32_t len_hint,
                                            uint8_t *d_ok, uint32_t *d_nbad, uint32_t *d_crc, uint32_t *d_hdr,
                                            uint32_t *d_pay, void *stream);

/* Region CRC of one long device buffer: *d_state_out = raw register after
 * feeding d_ptr[0, len) to `state_in` (val_crc32_update_state semantics;
 * finalize with ^0xFFFFFFFF). One launch at any length: windows up to 8
 * KiB are one 64-lane frame; longer ones are chunked over the whole machine
 * and folded inside the same launch through a 128-byte library-owned device
 * accumulator kept per stream (calls on one stream are ordered by it; calls
 * on different streams use different accumulators; hipStreamPerThread is
 * keyed per calling thread). The call runs on the stream's device (else the
 * device d_ptr lives on). */
val_status_t val_crc32_region_dev(const uint8_t *d_ptr, uint64_t len, uint32_t state_in, uint32_t *d_state_out,
                                  void *stream);
/* Scratch bytes the region call needs for a given length (informational). */
uint64_t val_crc32_region_scratch_bytes(uint64_t len);

/* ---- batch frames, host memory (synchronous; H2D + kernel + D2H, or the
 * CPU engine below val_gpu_host_batch_min_bytes) ---------------------------
 * base_len bounds every frame: off[i] + len[i] (+4 for verify) <= base_len,
 * else VAL_ERR_INVALID_ARG. off/len NULL = strided mode as above.
 * Frames travel H2D in chunks of whole frames on a copy stream while the
 * previous chunk is hashed (descriptor batches chunk when their offsets are
 * non-decreasing). A pinned `base` (val_gpu_host_alloc, hipHostMalloc or
 * hipHostRegister) is copied by DMA in place; pageable memory goes through
 * two internal pinned bounce buffers (host memcpy, val_gpu_host_copy_threads).
 * Mixed-length descriptor batches take the device-binned ragged path.   */
val_status_t val_crc32_frames_host(const uint8_t *base, uint64_t base_len, const uint64_t *off, const uint32_t *len,
                                   uint64_t stride, uint32_t flen, uint32_t n, uint32_t *crc, uint32_t *hdr);
val_status_t val_crc32_verify_frames_host(const uint8_t *base, uint64_t base_len, const uint64_t *off,
                                          const uint32_t *len, uint64_t stride, uint32_t flen, uint32_t n, uint8_t *ok,
                                          uint32_t *nbad);

/* Host batches whose CRC input totals fewer bytes than this are answered by
 * this library's CPU engine instead of the GPU, with identical outputs: a
 * host batch on the GPU pays a launch, a completion wait and PCIe for every
 * byte, and below the measured crossover one CPU core
 * is faster. -1 = VAL_GPU_HOST_BATCH_MIN_BYTES from the environment (read
 * once), else the built-in default, which depends on the batch's mean CRC
 * input per frame: 64 MiB from 4 KiB frames up, 32 MiB below (the getter
 * reports the former); 0 = always the GPU. Such batches need no device and
 * are counted by val_gpu_cpu_batch_count. */
void val_gpu_set_host_batch_min_bytes(int64_t bytes);
uint64_t val_gpu_host_batch_min_bytes(void);
/* The threshold a batch whose mean CRC input per frame is mean_len bytes is
 * held to (what val_crc32_frames_host applies to it). */
uint64_t val_gpu_host_batch_min_bytes_for(uint64_t mean_len);
uint64_t val_gpu_cpu_batch_count(void);
/* Threads the CPU engine uses for one such batch: the calling thread plus
 * threads - 1 helpers over byte-balanced frame ranges, at most one thread
 * per 4 MiB of CRC input (default 1), never more than the process's CPU
 * budget (its affinity set capped by the cgroup CPU quota). */
void val_gpu_set_host_cpu_threads(uint32_t threads);
/* The *_host_multi calls decide CPU or GPU once for the whole batch: below
 * val_gpu_host_batch_min_bytes() * T / N_eff bytes of CRC input, with T the
 * CPU engine's threads, the CPU engine answers it.
 * N_eff = N, the distinct devices the shards land on, for pinned input;
 * pageable input also passes through host bounce copies that all shards
 * share within the process's CPU budget, so N_eff = min(N, the measured
 * aggregate bounce-copy rate / one GPU's pageable rate). Returns that
 * threshold for `devices` devices and pageable input (_ex: pinned or not,
 * and a batch's mean CRC input per frame). */
uint64_t val_gpu_host_multi_min_bytes(int devices);
uint64_t val_gpu_host_multi_min_bytes_ex(int devices, int pinned, uint64_t mean_len);

/* Host-memory form of val_crc32_verify_frames_ex_dev (pay: n entries, nullable). */
val_status_t val_crc32_verify_frames_ex_host(const uint8_t *base, uint64_t base_len, const uint64_t *off,
                                             const uint32_t *len, uint64_t stride, uint32_t flen, uint32_t n,
                                             uint8_t *ok, uint32_t *nbad, uint32_t *pay);
/* The receiver's rolling CRC over frames 0..n-1 in order, stopping before the
 * first frame with ok[i] == 0 (ok nullable = all): for each frame
 * state = shift(state, pay_len[i]) ^ pay_state[i], i.e.
 * val_crc32_update_state(state, payload_i) without touching the bytes again.
 * The caller passes only in-order DATA frames (each payload starts where the
 * previous one ended); for a window that may hold duplicates, gaps or control
 * frames use val_crc32_fold_payload_states_at. *n_folded (nullable) = frames
 * folded. Host only (no GPU call). */
uint32_t val_crc32_fold_payload_states(uint32_t state, const uint32_t *pay_state, const uint32_t *pay_len,
                                       const uint8_t *ok, uint32_t n, uint32_t *n_folded);
/* The same fold with the receiver's ordering rule (reference
 * src/val_receiver.c:871-891): file_off[i] from val_frame_data_offsets
 * (val_wire.h). A frame is folded, and *written advanced by its payload,
 * only when it is a DATA frame with ok[i] != 0 whose effective offset
 * (file_off[i], or *written for VAL_FRAME_OFFSET_IMPLIED) equals *written;
 * duplicates (earlier offsets) and gaps (later ones) are skipped and the
 * frames after them are still judged one by one, as the receiver does.
 * *n_folded (nullable) = frames folded. Host only. */
uint32_t val_crc32_fold_payload_states_at(uint32_t state, const uint32_t *pay_state, const uint32_t *pay_len,
                                          const uint64_t *file_off, const uint8_t *ok, uint32_t n, uint64_t *written,
                                          uint32_t *n_folded);

/* ---- several GPUs in one process ----------------------------------------
 * The *_host batches above split into ndev shards (ndev <= 0: one per
 * visible device): contiguous frame ranges balanced by CRC-input bytes
 * (val_shard_frames), one host thread per shard running the single-device
 * path on device (shard % device count);
 * outputs are disjoint ranges of crc/hdr/ok, nbad is the sum. No collective
 * and no peer copies: frames are independent.                           */
val_status_t val_crc32_frames_host_multi(const uint8_t *base, uint64_t base_len, const uint64_t *off,
                                         const uint32_t *len, uint64_t stride, uint32_t flen, uint32_t n, uint32_t *crc,
                                         uint32_t *hdr, int ndev);
val_status_t val_crc32_verify_frames_host_multi(const uint8_t *base, uint64_t base_len, const uint64_t *off,
                                                const uint32_t *len, uint64_t stride, uint32_t flen, uint32_t n,
                                                uint8_t *ok, uint32_t *nbad, int ndev);
/* Raw register after feeding the host window data[0, len) to state_in, the
 * window cut into ndev 4 KiB-aligned byte ranges hashed on devices
 * (range % device count) and
 * folded with the GF(2) shift (val_crc32_update_state semantics). */
val_status_t val_crc32_region_host_multi(const void *data, uint64_t len, uint32_t state_in, uint32_t *state_out,
                                         int ndev);
/* [*start, *start + *count) = the frames shard `rank` of `world` owns:
 * contiguous, balanced by len[] (NULL: by count). Host only. */
void val_shard_frames(uint32_t n, const uint32_t *len, uint32_t world, uint32_t rank, uint32_t *start,
                      uint32_t *count);
/* Fold k partial raw states in order: state[0] carries the initial register,
 * state[i] (i >= 1) covers nbytes[i] bytes from a zero register.
 * acc = state[0]; acc = shift(acc, nbytes[i]) ^ state[i]. Host only. */
uint32_t val_crc32_fold_partials(const uint32_t *state, const uint64_t *nbytes, uint32_t k);

/* ---- pinned host staging ------------------------------------------------
 * Page-locked host memory for frame windows (e.g. the TX window staging
 * buffer of INTEGRATION.md section 3): the *_frames_host calls copy it by DMA
 * without a bounce. NULL on failure (val_gpu_last_error). */
void *val_gpu_host_alloc(size_t bytes);
void val_gpu_host_free(void *p);
/* Host threads one pageable-to-pinned copy of `bytes` uses when
 * `concurrent_copies` run at once (one per device in the *_host_multi
 * calls): one per 4 MiB, at most 8, and all copies together within the
 * process's CPU affinity set. */
uint32_t val_gpu_host_copy_threads(uint64_t bytes, uint32_t concurrent_copies);
/* Measurement of the pageable half of the host path, with no device work:
 * `copies` concurrent copy streams (as the shards of a *_host_multi call),
 * each copying `bytes` from resident pageable memory into its own bounce
 * buffer `reps` times through the library's own bounce copy (its thread
 * policy above). pinned_dst = 1: page-locked destinations (hipHostMalloc, as
 * the real bounce buffers); 0: malloc'd ones (no HIP runtime needed).
 * *gbs = copies * reps * bytes / the span from the common start to the last
 * copy's end, in GB/s. DESIGN.md section 1.3 folds it into the N-device
 * crossover. */
val_status_t val_gpu_host_copy_probe(uint32_t copies, uint64_t bytes, uint32_t reps, int pinned_dst, double *gbs);
/* Uniform batches whose frame groups do not fill the last round of the
 * persistent grid (e.g. 131,113 x 64 KiB frames: 8 rounds and 41 frames)
 * hash the frames past the last full round in pieces inside the same
 * launch (1-4 KiB pieces; 8 or 16 lanes per frame, frames of 8 KiB and more), instead of a
 * second launch. 1 / 0 switch it on / off, -1 = VAL_GPU_TAIL_PIECES (unset:
 * on). Speed only; results never change. _launches counts the launches that
 * used it. */
void val_gpu_set_tail_pieces(int enable);
uint64_t val_gpu_tail_piece_launches(void);
/* Wire bytes per H2D chunk of the *_frames_host calls; 0 = default (64 MiB).
 * Device memory use is two chunks. Speed and memory only; results never change. */
val_status_t val_gpu_set_host_chunk_bytes(size_t bytes);

/* ---- build and introspection --------------------------------------------
 * Diagnostic compile-time switches this library was built with, as a
 * space-separated list ("" for a product build). Switches that change
 * results can only be enabled in a VCRC_DIAG_BUILD, and such a build reports
 * "VCRC_DIAG_BUILD" here; tests/test_build.py asserts the in-tree library
 * reports nothing. */
const char *val_gpu_build_flags(void);
/* ---- introspection for benchmarks ---------------------------------------
 * Lanes per frame the library would pick for a given typical length. */
uint32_t val_gpu_lanes_per_frame(uint32_t typical_len);
/* Force the lanes-per-frame geometry (1,2,4,...,64) for later calls of this
 * process; 0 restores the automatic choice. Returns VAL_ERR_INVALID_ARG for
 * other values. Results never depend on it; only speed does. */
val_status_t val_gpu_set_lanes_per_frame(uint32_t lanes);
/* Rounds of each lane's input kept in flight ahead of the one being hashed:
 * 0, 1, 2 or 4 (copy and refill), or -2 / -3 (a ring of 2 or 3 rounds hashed
 * in their registers and refilled in place; 2 and 4 lanes per frame only,
 * others run 1); -1 = automatic: the 3-ring at 2 lanes, the 2-ring at 4 lanes
 * for frames under 1,600 B,
 * 1 otherwise. Speed only; results never change. */
val_status_t val_gpu_set_prefetch(int depth);
/* Mixed-length descriptor batches (len_hint 0) of at least this many frames
 * are binned by length on the device; smaller ones run uniform. -1 restores
 * VAL_GPU_RAGGED_MIN_FRAMES from the environment (read once), else 4096.
 * Speed only; results never change (tests pin the binned path with 1). */
void val_gpu_set_ragged_min_frames(int64_t frames);
uint32_t val_gpu_ragged_min_frames(void);
/* Streams of `device` that hold library scratch (region accumulator, ragged
 * binning, dynamic-tail queue); *evictions (nullable) = entries dropped so
 * far, least recently used first, once more than 64 streams held scratch.
 * Introspection for tests. */
uint32_t val_gpu_scratch_entries(int device, uint64_t *evictions);

#ifdef __cplusplus
}
#endif
#endif /* VAL_CRC32_GPU_H */
