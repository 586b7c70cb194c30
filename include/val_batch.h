/*
 * val_batch.h -- window batching of VAL's per-frame CRCs at the two hooks
 * the reference already exposes, with no change to its sources.
 *
 * The reference hashes one frame per call and sends it at once: TX frames
 * are built in the single send_buffer, CRC'd by val_internal_crc32 and
 * handed to transport.send (src/val_core.c:718-866, called W times per
 * window fill by src/val_sender.c:822-841); RX reads header, content and
 * trailer with three transport.recv calls and CRCs the frame in recv_buffer
 * (src/val_core.c:880-1073, called once per frame by the data loop of
 * src/val_receiver.c:801-1047). val_batch_attach() wraps a session's
 * val_config_t before val_session_create so that
 *
 *   TX: the CRC provider (val_config_t.crc32_provider, include/
 *       val_protocol.h:264-266) returns a placeholder for frames built in
 *       send_buffer, and the wrapped transport.send stages each frame in a
 *       window buffer instead of sending it. A window is flushed before the
 *       session next reads (the sender waits for ACKs after every window
 *       fill), when a control frame is sent, on transport.flush, or when the
 *       window buffer is full: the trailers of all staged frames come from
 *       ONE val_crc32_frames_host call, are written little-endian, and the
 *       frames go to the application's transport in order. The wire is the
 *       reference's, byte for byte; only the time of sending moves to the
 *       end of the window fill.
 *   RX: (recv_polls, below) the wrapped transport.recv reads ahead: the
 *       frame the session asked for (over as many short reads as the
 *       transport returns, within the session's timeout, measured with
 *       config->system.get_ticks_ms) plus every further frame the transport
 *       already holds (polled with a zero timeout while polls return bytes),
 *       up to the window limits; no byte read is ever dropped (a frame cut
 *       off by a poll finishes in the next read-ahead and is delivered
 *       unbatched). It computes their CRCs with ONE val_crc32_frames_host
 *       call. It hands bytes to the
 *       session exactly as asked; when a frame's header and content were
 *       delivered to recv_buffer in place and its trailer after them, the
 *       provider call that follows (src/val_core.c:964) is answered with
 *       that frame's batch CRC. Every other provider call (resume windows,
 *       frames split across read-aheads) is computed directly.
 *
 * When batching pays (VAL_BATCH_AUTO, the default): a batch makes the CRC
 * faster only when it is large enough to run on the GPU. Below the host-batch
 * crossover (val_gpu_host_batch_min_bytes) a batch runs on the same CPU
 * engine the provider uses per frame, so batching cannot speed the CRC up; it
 * only moves frames in time (the sender's frames wait for the end of the
 * window fill, the receiver reads ahead). Measured on the reference's own
 * loopback, that moved the transfer rate by -24% to +14% against the plain
 * provider depending on window and direction. So in
 * AUTO a direction batches only when a device was present at attach and
 * its largest possible batch,
 * min(max_bytes, window_cap_packets x packet_size), reaches the crossover
 * (checked at every window, so val_gpu_set_host_batch_min_bytes takes effect
 * at once); otherwise TX frames get their trailer from the provider and go
 * out at once, and RX reads only the frame the session asked for, whose
 * check the provider computes. ALWAYS batches regardless (coalesce_send
 * implies it for TX).
 *
 * Reading ahead means polling the transport with a zero timeout. The
 * reference's contract does not define timeout 0 (the reference itself never
 * passes it, src/val_core.c:31) and its own TCP example blocks forever on it
 * (examples/tcp/common/tcp_util.c:383), which would deadlock a read-ahead at
 * the end of every window. So RX reads ahead only when the application says
 * its recv polls (recv_polls = 1). Such a poll must also be cheap: a
 * condition-variable wait on an already expired deadline took ~70 us per
 * empty poll in our harness and added that to every read-ahead.
 *
 * A batch the GPU path fails is computed on the CPU engine instead
 * (batch_fallbacks): like the provider, the batcher never fails a session
 * over a device error.
 *
 * Transport failures. A deferred frame's send happens at the window flush,
 * not in the session's send call: the session counts a staged DATA frame as
 * sent when it is staged (its `sent` metrics, src/val_core.c:844), and a
 * send that fails at the flush ends that window (the frames after it are not
 * sent: tx_unsent) and is returned, once, by the hook call that flushed: the
 * session's next transport.recv (its ACK wait for that window, so
 * val_send_files returns VAL_ERR_IO within that window, with detail
 * RECV_FAILED where the reference records SEND_FAILED), or the send that
 * stages a control frame or overflows the window (SEND_FAILED). A flush from
 * transport.flush, which has no status, is reported by the next send or
 * recv. stats.status names the failure. After it has been reported the
 * batcher works again: a later val_send_files on the same session runs as on
 * the bare transport.
 *
 * RX answers. The provider answers a call from an RX batch only when its
 * buffer is the attached recv_buffer, right after the frame's trailer was
 * delivered, with the frame's length, and with recv_buffer still holding the
 * frame's 8 header bytes and last CRC-input bytes; anything else (a resume
 * window read into recv_buffer, src/val_core.c:431-436) is computed directly
 * (arm_rejects). A header announcing content beyond the MTU stops read-ahead
 * (the stream's frame boundaries are lost; the session rejects that frame):
 * the session's reads pass straight through until they have taken one whole
 * frame the way the session reads frames (header, the content it announces,
 * trailer), which puts this parser back on the session's frame boundaries;
 * read-ahead resumes there (resyncs).
 *
 * Memory. A direction allocates its window (max_bytes, pinned when a device
 * was present at attach) when it first batches; until then the RX ring holds
 * one frame. A batcher with both directions OFF never starts the HIP runtime.
 *
 * The application keeps its own transport and provider semantics: the
 * wrapped hooks call the ones in the config at attach time (a NULL provider
 * means this library's val_gpu_crc32_provider). Batches below the host-batch
 * crossover run on the CPU engine, larger ones on the GPU;
 * VAL_GPU_HOST_BATCH_MIN_BYTES=0 sends every window to the GPU.
 */
#ifndef VAL_BATCH_H
#define VAL_BATCH_H

#include <stddef.h>
#include <stdint.h>

#include "val_errors.h"
#include "val_protocol.h"

#ifdef __cplusplus
extern "C" {
#endif

#define VAL_BATCH_OFF 0     /* the reference's behaviour: the provider per frame */
#define VAL_BATCH_AUTO 1    /* batch when a batch can reach the GPU (see above) */
#define VAL_BATCH_ALWAYS 2  /* batch every window */

typedef struct {
    uint32_t max_frames;  /* frames per batch, TX and RX (0 = 65,535) */
    size_t max_bytes;     /* wire bytes per batch (0 = window_cap_packets x packet_size within [16, 256] MiB;
                             at least one MTU) */
    int tx;               /* VAL_BATCH_*: defer TX trailers to window batches */
    int rx;               /* VAL_BATCH_*: read ahead and hash RX frames in batches */
    int coalesce_send;    /* 1: one transport.send per flushed window (0: one per frame, as the reference) */
    int recv_polls;       /* 1: transport.recv with timeout 0 returns at once (nothing there: *received = 0), as a
                             non-blocking socket read does; RX reads ahead only then. 0 (default): the reference's
                             contract, where timeout 0 may block (its TCP example waits forever): RX reads only
                             the frame the session asked for, and its checks come from the provider */
} val_batch_opts_t;

typedef struct {
    uint64_t tx_frames;          /* frames passed to the application's transport.send */
    uint64_t tx_batched_frames;  /* of those, trailers computed in a window batch */
    uint64_t tx_batches;         /* window batches (one frames_host call each) */
    uint64_t tx_max_batch;       /* most frames in one TX batch */
    uint64_t rx_frames;          /* complete frames read ahead */
    uint64_t rx_batches;         /* RX batches (one frames_host call each) */
    uint64_t rx_max_batch;       /* most frames in one RX batch */
    uint64_t rx_batched_answers; /* provider calls answered from an RX batch */
    uint64_t direct_answers;     /* provider calls computed directly (resume windows, split frames) */
    uint64_t batch_fallbacks;    /* batches the GPU path failed and the CPU engine computed (the provider's policy) */
    int32_t status;              /* the most recent transport or batch failure (VAL_OK if none) */
    uint64_t failures;           /* transport or batch failures (each reported once to the session, see below) */
    uint64_t tx_unsent;          /* staged frames never sent: they followed a failed send in their window */
    uint64_t arm_rejects;        /* same-length provider calls on recv_buffer whose bytes were not the armed frame
                                    (computed directly) */
    uint64_t resyncs;            /* read-ahead resumed after an oversize header (the session's reads framed again) */
} val_batch_stats_t;

typedef struct val_batch val_batch_t;

/* Wrap cfg->transport and cfg->crc32_provider (cfg->buffers.send_buffer,
 * recv_buffer and packet_size must be set; the two buffers must differ and
 * not belong to another attached config: VAL_ERR_INVALID_ARG otherwise).
 * opts may be NULL (defaults: VAL_BATCH_AUTO both ways; tx/rx outside
 * VAL_BATCH_OFF..ALWAYS: VAL_ERR_INVALID_ARG). Attach before
 * val_session_create (the session copies the config); call val_batch_detach
 * after val_session_destroy. Up to 256 attached configs per process. */
val_status_t val_batch_attach(val_config_t *cfg, const val_batch_opts_t *opts, val_batch_t **out);
/* Send the staged TX window now (the wrapped hooks do this themselves). */
val_status_t val_batch_flush(val_batch_t *b);
void val_batch_get_stats(const val_batch_t *b, val_batch_stats_t *out);
/* Flush, restore cfg's hooks and free the batcher. */
void val_batch_detach(val_batch_t *b);
/* The provider val_batch_attach installs (crc32_func_t): a placeholder for a
 * frame in an attached send_buffer, the batch CRC of a frame delivered in
 * place to an attached recv_buffer, else val_gpu_crc32_provider semantics. */
uint32_t val_batch_crc32_provider(uint32_t seed, const void *buf, size_t len);

#ifdef __cplusplus
}
#endif

#endif /* VAL_BATCH_H */
