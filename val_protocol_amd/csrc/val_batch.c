/*
 * val_batch.c -- window batching of VAL's per-frame CRCs through the
 * reference's own hooks (include/val_batch.h). TX: placeholder trailers from
 * the provider, frames staged by the wrapped transport.send and hashed in
 * one val_crc32_frames_host call per window (reference src/val_core.c:
 * 828-835, src/val_sender.c:822-841). RX: the wrapped transport.recv reads
 * ahead whole frames, hashes them in one call, and the provider answers the
 * session's per-frame check (src/val_core.c:963-974) from that batch.
 */
#include "val_batch.h"

#include <stdlib.h>
#include <string.h>

#include "val_crc32_gpu.h"
#include "val_wire.h"

#define VB_MAX_ATTACHED 256
#define VB_MIN_DEFAULT_BYTES ((size_t)16u << 20)   /* default max_bytes: the window, within these */
#define VB_MAX_DEFAULT_BYTES ((size_t)256u << 20)
#define VB_DEFAULT_FRAMES 65535u

typedef struct {
    uint64_t off;  /* in the window / ring buffer */
    uint32_t len;  /* CRC input = wire - 4 */
    uint32_t crc;  /* batch CRC (RX), or the trailer to write (TX) */
    uint8_t need;  /* TX: trailer comes from the batch */
} vb_frame_t;

struct val_batch {
    val_config_t *cfg;
    /* the application's hooks, called by the wrappers */
    int (*u_send)(void *, const void *, size_t);
    int (*u_recv)(void *, void *, size_t, size_t *, uint32_t);
    int (*u_is_connected)(void *);
    void (*u_flush)(void *);
    void *u_io;
    crc32_func_t u_provider;
    val_batch_opts_t opt;
    const uint8_t *send_buffer, *recv_buffer;
    size_t mtu;
    uint32_t win_cap;        /* the config's window cap in frames (0 in the config = 1, src/val_core.c:1755) */
    int pinned;              /* allocate windows pinned (a device is present) */
    int tx_pinned, rx_pinned; /* how each window buffer was allocated */
    int err;                 /* a failure no hook call has reported to the session yet (transport.flush has no
                                status): the next send or recv reports it, once */
    /* TX window: allocated when TX first batches */
    uint8_t *tx;
    size_t tx_cap;
    size_t tx_used;
    vb_frame_t *txf;
    uint32_t tx_n;
    size_t tx_pending;  /* CRC input of the frame whose placeholder was just returned (0: none) */
    /* RX ring: bytes [r_head, r_len) not yet handed to the session */
    uint8_t *rx;
    size_t rx_cap;  /* the ring's bytes: one frame until RX first batches, then max_bytes */
    size_t r_head, r_len;
    vb_frame_t *rxf;
    uint32_t rx_n, rx_cur;  /* complete frames in the ring; the one being delivered */
    uint64_t r_base;        /* stream position of rx[0] */
    /* stream parse state: bytes still owed by the transport for the frame in
       progress (0 = at a frame boundary), and whether a header is partial */
    size_t owe;
    uint8_t hdr_part[8];
    size_t hdr_have;
    uint32_t cur_len;  /* CRC input of the frame in progress (its header is complete) */
    uint32_t (*ticks)(void);  /* the config's clock (val_config_t.system.get_ticks_ms), for read deadlines */
    int raw;  /* a header announced content beyond the MTU: read-ahead stops until the session's own reads
                 show it at a frame boundary again (rs_*) */
    int rs_seg;             /* while raw: the segment the session is reading (0 header, 1 content, 2 trailer;
                               -1 unknown) */
    size_t rs_left;         /* its bytes still to come */
    uint8_t rs_hdr[VAL_WIRE_HEADER_SIZE];
    /* delivery of frame rx_cur into recv_buffer in place */
    size_t cur_matched;
    int armed;
    uint32_t armed_len, armed_crc;
    uint8_t armed_head[VAL_WIRE_HEADER_SIZE];  /* the armed frame's header and last CRC-input bytes: the */
    uint8_t armed_tail[8];                      /* provider answers from the batch only for these bytes */
    uint32_t armed_tail_n;
    val_batch_stats_t st;
    /* per-frame arrays, allocated with the first window buffer */
    uint32_t *crc_tmp;
    uint64_t *off_tmp;
    uint32_t *len_tmp;
};

/* The attached sessions: a slot's buffers are compared without touching its
 * batcher, so a provider call never dereferences another session's batcher
 * (which its own thread may be detaching and freeing). A buffer that matches
 * is the calling session's own, and so is the batcher in that slot. */
static val_batch_t *g_reg[VB_MAX_ATTACHED];
static const void *g_buf[2][VB_MAX_ATTACHED];  /* [0]: send_buffer, [1]: recv_buffer */
static int g_hwm;  /* slots [0, g_hwm) have been used: the provider scans only those */

/* The slot this thread last found per direction: a session's thread calls the
 * provider on the same two buffers frame after frame, so the scan (up to 256
 * slots once many sessions are attached) runs once per thread and session.
 * The hint is only a starting guess: a slot matches only if it holds this very
 * buffer now. */
static __thread int t_slot_hint[2] = {-1, -1};

/* The attached batcher whose send_buffer (*rx = 0) or recv_buffer (*rx = 1)
 * is buf, or NULL. */
static val_batch_t *vb_find(const void *buf, int *rx)
{
    if (!buf) return NULL;  /* a free slot's buffers read NULL */
    for (int d = 0; d < 2; d++) {
        const int h = t_slot_hint[d];
        if (h >= 0 && __atomic_load_n(&g_buf[d][h], __ATOMIC_ACQUIRE) == buf) {
            *rx = d;
            return __atomic_load_n(&g_reg[h], __ATOMIC_ACQUIRE);
        }
    }
    const int hwm = __atomic_load_n(&g_hwm, __ATOMIC_ACQUIRE);
    for (int i = 0; i < hwm; i++)
        for (int d = 0; d < 2; d++)
            if (__atomic_load_n(&g_buf[d][i], __ATOMIC_ACQUIRE) == buf) {
                t_slot_hint[d] = i;
                *rx = d;
                return __atomic_load_n(&g_reg[i], __ATOMIC_ACQUIRE);
            }
    return NULL;
}

static val_batch_t *vb_lookup(const void *buf, int rx)
{
    int d = 0;
    val_batch_t *b = vb_find(buf, &d);
    return d == rx ? b : NULL;
}

static uint32_t vb_direct(val_batch_t *b, uint32_t seed, const void *buf, size_t len)
{
    if (b) b->st.direct_answers++;
    crc32_func_t p = b && b->u_provider ? b->u_provider : val_gpu_crc32_provider;
    return p(seed, buf, len);
}

static void vb_fail(val_batch_t *b, val_status_t st)
{
    b->st.status = st;
    b->st.failures++;
}

/* The host-batch crossover for this session's frames: their mean CRC input
 * is about one MTU, so AUTO decides as val_crc32_frames_host will for the
 * batch it would send (val_gpu_host_batch_min_bytes_for). */
static int vb_engaged(const val_batch_t *b, int mode)
{
    if (mode == VAL_BATCH_ALWAYS) return 1;
    if (mode != VAL_BATCH_AUTO) return 0;
    if (!b->pinned) return 0;  /* no device at attach: every batch would run on the CPU engine */
    uint64_t ub = (uint64_t)b->win_cap * b->mtu;
    if (ub > b->opt.max_bytes) ub = b->opt.max_bytes;
    return ub >= val_gpu_host_batch_min_bytes_for(b->mtu - VAL_WIRE_TRAILER_SIZE);
}

static void *vb_alloc(const val_batch_t *b, size_t n, int *pinned)
{
    void *p = b->pinned ? val_gpu_host_alloc(n) : NULL;
    *pinned = p != NULL;
    return p ? p : malloc(n);
}

static void vb_free(void *p, int pinned)
{
    if (!p) return;
    if (pinned) val_gpu_host_free(p);
    else free(p);
}

/* The per-frame arrays both directions share, on first use. */
static int vb_frames_ready(val_batch_t *b)
{
    if (b->crc_tmp) return 1;
    const uint32_t nf = b->opt.max_frames;
    uint32_t *c = (uint32_t *)calloc(nf, sizeof(uint32_t));
    uint64_t *o = (uint64_t *)calloc(nf, sizeof(uint64_t));
    uint32_t *l = (uint32_t *)calloc(nf, sizeof(uint32_t));
    if (!c || !o || !l) {
        free(c);
        free(o);
        free(l);
        return 0;
    }
    b->crc_tmp = c;
    b->off_tmp = o;
    b->len_tmp = l;
    return 1;
}

/* The TX window, allocated when TX first batches (a session whose windows
 * never reach the crossover pins nothing). 0: no memory; the frame is then
 * hashed by the provider and sent at once. */
static int vb_tx_ready(val_batch_t *b)
{
    if (b->tx) return 1;
    if (!vb_frames_ready(b)) return 0;
    vb_frame_t *f = (vb_frame_t *)calloc(b->opt.max_frames, sizeof(vb_frame_t));
    uint8_t *w = f ? (uint8_t *)vb_alloc(b, b->opt.max_bytes, &b->tx_pinned) : NULL;
    if (!w) {
        free(f);
        return 0;
    }
    b->txf = f;
    b->tx = w;
    b->tx_cap = b->opt.max_bytes;
    return 1;
}

/* The RX ring grown from one frame to a batch window when RX first batches;
 * called only with the ring empty. 0: no memory (this fill reads one frame). */
static int vb_rx_ready(val_batch_t *b)
{
    if (b->rxf && b->rx_cap >= b->opt.max_bytes) return 1;
    if (!vb_frames_ready(b)) return 0;
    vb_frame_t *f = (vb_frame_t *)calloc(b->opt.max_frames, sizeof(vb_frame_t));
    int pinned = 0;
    uint8_t *r = f ? (uint8_t *)vb_alloc(b, b->opt.max_bytes, &pinned) : NULL;
    if (!r) {
        free(f);
        return 0;
    }
    memcpy(r, b->rx, b->r_len);  /* bytes of a frame in progress (none at a fill's start) */
    vb_free(b->rx, b->rx_pinned);
    b->rx = r;
    b->rx_pinned = pinned;
    b->rx_cap = b->opt.max_bytes;
    b->rxf = f;
    return 1;
}

static int vb_tx_engaged(const val_batch_t *b)
{
    return b->opt.tx && (b->opt.coalesce_send || vb_engaged(b, b->opt.tx));
}

/* CRCs of frames f[0..n) of buf in one host batch call. */
static val_status_t vb_hash(val_batch_t *b, const uint8_t *buf, size_t used, vb_frame_t *f, uint32_t n, int only_needed)
{
    uint32_t k = 0;
    for (uint32_t i = 0; i < n; i++)
        if (!only_needed || f[i].need) {
            b->off_tmp[k] = f[i].off;
            b->len_tmp[k] = f[i].len;
            k++;
        }
    if (!k) return VAL_OK;
    const val_status_t st = val_crc32_frames_host(buf, used, b->off_tmp, b->len_tmp, 0, 0, k, b->crc_tmp, NULL);
    if (st == VAL_ERR_INVALID_ARG) return st;  /* our own descriptors: a bug, not a device failure */
    if (st != VAL_OK) {
        /* the provider's failure policy (it has no error channel):
           a batch the GPU could not take is computed on the CPU engine */
        for (uint32_t i = 0; i < k; i++)
            b->crc_tmp[i] = val_crc32_cpu_update_state(0xFFFFFFFFu, buf + b->off_tmp[i], b->len_tmp[i], 0) ^ 0xFFFFFFFFu;
        b->st.batch_fallbacks++;
    }
    k = 0;
    for (uint32_t i = 0; i < n; i++)
        if (!only_needed || f[i].need) f[i].crc = b->crc_tmp[k++];
    return VAL_OK;
}

/* ---- TX ---------------------------------------------------------------- */
/* Send the staged window: trailers from one batch, then the frames in order.
 * A transport send that fails ends the window there: the frames after it are
 * not sent (tx_unsent), as the reference's sender stops at the frame whose
 * send failed (src/val_core.c:835-842, src/val_sender.c:835-840). The
 * failure is returned to this call only (the caller reports it to the
 * session once); the batcher itself stays usable for later transfers. */
static val_status_t vb_flush_tx(val_batch_t *b)
{
    if (!b->tx_n) return VAL_OK;
    uint32_t need = 0;
    for (uint32_t i = 0; i < b->tx_n; i++) need += b->txf[i].need;
    val_status_t st = VAL_OK;
    uint32_t sent = 0;
    if (need) {
        st = vb_hash(b, b->tx, b->tx_used, b->txf, b->tx_n, 1);
        if (st == VAL_OK) {
            b->st.tx_batches++;
            b->st.tx_batched_frames += need;
            if (need > b->st.tx_max_batch) b->st.tx_max_batch = need;
            for (uint32_t i = 0; i < b->tx_n; i++)
                if (b->txf[i].need) {
                    uint8_t *t = b->tx + b->txf[i].off + b->txf[i].len;
                    const uint32_t c = b->txf[i].crc;
                    t[0] = (uint8_t)c;
                    t[1] = (uint8_t)(c >> 8);
                    t[2] = (uint8_t)(c >> 16);
                    t[3] = (uint8_t)(c >> 24);
                }
        } else {
            vb_fail(b, st);
        }
    }
    if (st == VAL_OK) {
        if (b->opt.coalesce_send) {
            if (b->u_send(b->u_io, b->tx, b->tx_used) == (int)b->tx_used) sent = b->tx_n;
            else vb_fail(b, st = VAL_ERR_IO);
        } else {
            for (; sent < b->tx_n; sent++) {
                const size_t wl = (size_t)b->txf[sent].len + VAL_WIRE_TRAILER_SIZE;
                if (b->u_send(b->u_io, b->tx + b->txf[sent].off, wl) != (int)wl) {
                    vb_fail(b, st = VAL_ERR_IO);
                    break;
                }
            }
        }
    }
    b->st.tx_frames += sent;
    b->st.tx_unsent += b->tx_n - sent;
    b->tx_n = 0;
    b->tx_used = 0;
    return st;
}

/* A failure the session has not been told about (from transport.flush):
 * reported by this call, once. */
static int vb_take_err(val_batch_t *b)
{
    if (!b->err) return 0;
    b->err = 0;
    return 1;
}

static int vb_send(void *ctx, const void *data, size_t len)
{
    val_batch_t *b = (val_batch_t *)ctx;
    const size_t pending = b->tx_pending;
    b->tx_pending = 0;
    if (vb_take_err(b)) return -1;
    /* the provider returned a placeholder for exactly this frame (and made
       sure the window exists) */
    const int placeholder = data == (const void *)b->send_buffer && len >= VAL_WIRE_TRAILER_SIZE &&
                            pending == len - VAL_WIRE_TRAILER_SIZE && b->tx;
    if (!b->opt.tx || len < VAL_WIRE_HEADER_SIZE + VAL_WIRE_TRAILER_SIZE || len > b->opt.max_bytes ||
        (!placeholder && b->tx_n == 0 && (!vb_tx_engaged(b) || !vb_tx_ready(b)))) {
        /* not a frame this batcher stages: send the window before it, then it */
        if (vb_flush_tx(b) != VAL_OK) return -1;
        const int rc = b->u_send(b->u_io, data, len);
        if (rc == (int)len) b->st.tx_frames++;
        else vb_fail(b, VAL_ERR_IO);
        return rc;
    }
    if (b->tx_n == b->opt.max_frames || b->tx_used + len > b->tx_cap)
        if (vb_flush_tx(b) != VAL_OK) return -1;
    vb_frame_t *f = &b->txf[b->tx_n++];
    f->off = b->tx_used;
    f->len = (uint32_t)(len - VAL_WIRE_TRAILER_SIZE);
    f->need = (uint8_t)placeholder;
    memcpy(b->tx + b->tx_used, data, len);
    b->tx_used += len;
    const uint8_t type = ((const uint8_t *)data)[0];
    /* only DATA frames wait for the rest of their window: a control frame
       (ACK, DONE, EOT, ...) goes out at once with everything before it */
    if (type != VAL_PKT_DATA && vb_flush_tx(b) != VAL_OK) return -1;
    return (int)len;
}

static void vb_flush_hook(void *ctx)
{
    val_batch_t *b = (val_batch_t *)ctx;
    if (vb_flush_tx(b) != VAL_OK) b->err = 1;  /* flush has no status: the next send or recv reports it */
    if (b->u_flush) b->u_flush(b->u_io);
}

static int vb_is_connected(void *ctx)
{
    val_batch_t *b = (val_batch_t *)ctx;
    return b->u_is_connected ? b->u_is_connected(b->u_io) : 1;
}

/* ---- RX ---------------------------------------------------------------- */
/* Read up to n bytes into dst from the application's transport within
 * timeout (its recv may return fewer); returns the bytes read or -1. */
static long vb_read(val_batch_t *b, uint8_t *dst, size_t n, uint32_t timeout_ms)
{
    size_t got = 0;
    const int rc = b->u_recv(b->u_io, dst, n, &got, timeout_ms);
    if (rc < 0) return -1;
    return (long)(got > n ? n : got);
}

static size_t vb_content_max(const val_batch_t *b)
{
    return b->mtu - VAL_WIRE_HEADER_SIZE - VAL_WIRE_TRAILER_SIZE;
}

/* Refill the empty ring. Batching (RX engaged, on a transport that polls,
 * recv_polls): the frame in progress (or the next one), for which the
 * transport is given up to timeout_ms as the session would give it (over as
 * many partial reads as it takes), then every further byte it already holds
 * (zero-timeout polls, until one returns nothing); the complete frames that
 * began in this ring are hashed in one batch. Not batching: only until the
 * `want` bytes the session asked for are in, so each of the session's reads
 * waits no longer than it would on the bare transport (its header read does
 * not wait for the content). Returns 0, or -1 on a transport error. */
static int vb_fill(val_batch_t *b, uint32_t timeout_ms, size_t want)
{
    b->r_base += b->r_len;
    b->r_head = b->r_len = 0;
    b->rx_n = b->rx_cur = 0;
    const uint32_t t0 = b->ticks ? b->ticks() : 0u;
    int eng = b->opt.recv_polls && vb_engaged(b, b->opt.rx);
    if (eng && !vb_rx_ready(b)) eng = 0;
    const size_t cap = b->rx_cap;
    const uint32_t lim = eng ? b->opt.max_frames : 1u;
    uint32_t nread = 0;
    /* a frame carried over from the previous ring is delivered, not batched */
    int whole = b->hdr_have == 0 && b->owe == 0;
    uint64_t fstart = 0;
    int first = 1, attempted = 0;
    for (;;) {
        /* past the first frame every read is a zero-timeout poll: only on a
           transport that says it polls (val_batch_opts_t.recv_polls) */
        if (!first && !b->opt.recv_polls) break;
        if (!eng && b->r_len >= want) break;
        uint32_t budget = 0;  /* frames read ahead: only what is there */
        if (first) {
            const uint32_t el = b->ticks ? b->ticks() - t0 : 0u;
            if (attempted && el >= timeout_ms) break;  /* the session's time is up: it gets what there is */
            /* as val_recv_full (src/val_core.c:29-31): never 0 once the
               session gave a timeout, since a transport may block on 0 */
            budget = timeout_ms > el ? timeout_ms - el : (timeout_ms ? 1u : 0u);
            attempted = 1;
        }
        if (b->owe == 0) {  /* the header */
            if (b->hdr_have == 0) {
                if (nread >= lim || cap - b->r_len < b->mtu) break;
                fstart = b->r_len;
            }
            const long g = vb_read(b, b->hdr_part + b->hdr_have, VAL_WIRE_HEADER_SIZE - b->hdr_have, budget);
            if (g < 0) return -1;
            memcpy(b->rx + b->r_len, b->hdr_part + b->hdr_have, (size_t)g);
            b->r_len += (size_t)g;
            b->hdr_have += (size_t)g;
            if (b->hdr_have < VAL_WIRE_HEADER_SIZE) {
                if (g > 0 && (!first || budget > 0)) continue;  /* partial read: more may be there */
                break;
            }
            const size_t content = (size_t)b->hdr_part[2] | (size_t)b->hdr_part[3] << 8;
            if (content > vb_content_max(b)) {
                /* the session will reject it (src/val_core.c:915-921); the
                   stream has no trustworthy boundaries until it goes quiet */
                b->raw = 1;
                b->rs_seg = -1;
                b->hdr_have = 0;
                break;
            }
            b->cur_len = (uint32_t)(VAL_WIRE_HEADER_SIZE + content);
            b->owe = content + VAL_WIRE_TRAILER_SIZE;
            if (!eng && b->r_len >= want) break;
        }
        const long r = vb_read(b, b->rx + b->r_len, b->owe, budget);
        if (r < 0) return -1;
        b->r_len += (size_t)r;
        b->owe -= (size_t)r;
        if (b->owe) {
            if (!eng && b->r_len >= want) break;
            if (r > 0 && (!first || budget > 0)) continue;
            break;
        }
        nread += whole;
        if (whole && eng) {  /* complete, and every byte of it is in this ring */
            vb_frame_t *f = &b->rxf[b->rx_n++];
            f->off = fstart;
            f->len = b->cur_len;
            f->need = 1;
        }
        b->hdr_have = 0;
        whole = 1;
        first = 0;
    }
    if (b->rx_n) {
        const val_status_t st = vb_hash(b, b->rx, b->r_len, b->rxf, b->rx_n, 0);
        if (st != VAL_OK) {
            vb_fail(b, st);
            b->rx_n = 0;  /* the session's checks are then computed directly */
        } else {
            b->st.rx_batches++;
            b->st.rx_frames += b->rx_n;
            if (b->rx_n > b->st.rx_max_batch) b->st.rx_max_batch = b->rx_n;
        }
    }
    return 0;
}

/* Bytes [pos, pos + n) of the ring went to dst: track whether frame rx_cur
 * is being delivered to recv_buffer in place, and arm its CRC for the
 * provider call that follows its trailer. */
static void vb_track(val_batch_t *b, size_t pos, size_t n, const uint8_t *dst)
{
    b->armed = 0;
    while (n && b->rx_cur < b->rx_n) {
        vb_frame_t *f = &b->rxf[b->rx_cur];
        const size_t fs = (size_t)f->off, fe = fs + f->len + VAL_WIRE_TRAILER_SIZE;
        if (pos >= fe) {
            b->rx_cur++;
            b->cur_matched = 0;
            continue;
        }
        if (pos < fs) {  /* bytes before this frame (a partial tail of an earlier one) */
            const size_t skip = fs - pos < n ? fs - pos : n;
            pos += skip;
            dst += skip;
            n -= skip;
            continue;
        }
        const size_t take = fe - pos < n ? fe - pos : n;
        /* CRC-input bytes of this piece that landed at recv_buffer + (pos - fs) */
        const size_t ce = fs + f->len;
        if (pos < ce) {
            const size_t cn = (ce - pos < take) ? ce - pos : take;
            if (dst == b->recv_buffer + (pos - fs)) b->cur_matched += cn;
        }
        pos += take;
        dst += take;
        n -= take;
        if (pos == fe) {
            if (b->cur_matched == f->len) {
                b->armed = 1;
                b->armed_len = f->len;
                b->armed_crc = f->crc;
                /* f->len >= 8: every frame has its header */
                memcpy(b->armed_head, b->rx + fs, VAL_WIRE_HEADER_SIZE);
                b->armed_tail_n = f->len - VAL_WIRE_HEADER_SIZE < 8u ? f->len - VAL_WIRE_HEADER_SIZE : 8u;
                memcpy(b->armed_tail, b->rx + fs + f->len - b->armed_tail_n, b->armed_tail_n);
            }
            b->rx_cur++;
            b->cur_matched = 0;
        }
    }
}

/* Passthrough after an oversize header: follow the session's own reads. It
 * reads a frame as header (8 bytes), then exactly the content its header
 * announces, then the 4-byte trailer (src/val_core.c:893-945), over as many
 * partial reads as the transport returns. Once its reads have taken one whole
 * frame that way, this parser and the session agree where frames start
 * again, and read-ahead resumes at the next frame. Reads of any other shape
 * (a rejected header, a timeout mid-frame) restart the match at the session's
 * next header read. */
static void vb_raw_track(val_batch_t *b, const uint8_t *buf, size_t asked, size_t got)
{
    if (b->rs_seg < 0 || asked != b->rs_left) {
        if (asked != VAL_WIRE_HEADER_SIZE) {
            b->rs_seg = -1;
            return;
        }
        b->rs_seg = 0;
        b->rs_left = VAL_WIRE_HEADER_SIZE;
    }
    if (b->rs_seg == 0) memcpy(b->rs_hdr + (VAL_WIRE_HEADER_SIZE - b->rs_left), buf, got);
    b->rs_left -= got;
    if (b->rs_left) return;
    if (b->rs_seg == 0) {
        const size_t content = (size_t)b->rs_hdr[2] | (size_t)b->rs_hdr[3] << 8;
        if (content > vb_content_max(b)) {
            b->rs_seg = -1;
            return;
        }
        b->rs_seg = content ? 1 : 2;
        b->rs_left = content ? content : VAL_WIRE_TRAILER_SIZE;
    } else if (b->rs_seg == 1) {
        b->rs_seg = 2;
        b->rs_left = VAL_WIRE_TRAILER_SIZE;
    } else {  /* a whole frame as the session read it: the next byte starts a frame */
        b->raw = 0;
        b->owe = b->hdr_have = 0;
        b->st.resyncs++;
    }
}

static int vb_recv(void *ctx, void *buffer, size_t size, size_t *received, uint32_t timeout_ms)
{
    val_batch_t *b = (val_batch_t *)ctx;
    if (received) *received = 0;
    if (size == 0) return 0;
    if (vb_take_err(b)) return -1;
    /* the session is about to wait: its staged window goes out first (a
       failed send is this call's error: the session's ACK wait fails with
       VAL_ERR_IO in the window whose frame was lost) */
    if (vb_flush_tx(b) != VAL_OK) return -1;
    if (!b->opt.rx) return b->u_recv(b->u_io, buffer, size, received, timeout_ms);
    if (b->r_head == b->r_len) {
        if (b->raw) {
            b->armed = 0;
            size_t got = 0;
            const int rc = b->u_recv(b->u_io, buffer, size, &got, timeout_ms);
            if (received) *received = got;
            if (rc >= 0) vb_raw_track(b, (const uint8_t *)buffer, size, got > size ? size : got);
            return rc;
        }
        if (vb_fill(b, timeout_ms, size) < 0) return -1;
    }
    size_t n = b->r_len - b->r_head;
    if (n > size) n = size;
    if (n) {
        memcpy(buffer, b->rx + b->r_head, n);
        vb_track(b, b->r_head, n, (const uint8_t *)buffer);
        b->r_head += n;
    }
    if (received) *received = n;
    return 0;
}

/* ---- the provider ------------------------------------------------------ */
/* Whether the bytes at buf are the armed frame: its header and its last CRC-
 * input bytes, which any other content put in recv_buffer since (a resume
 * window read there, src/val_core.c:431-436, another frame) changes. */
static int vb_arm_matches(const val_batch_t *b, const uint8_t *buf, size_t len)
{
    return memcmp(buf, b->armed_head, VAL_WIRE_HEADER_SIZE) == 0 &&
           memcmp(buf + len - b->armed_tail_n, b->armed_tail, b->armed_tail_n) == 0;
}

uint32_t val_batch_crc32_provider(uint32_t seed, const void *buf, size_t len)
{
    int rx = 0;
    val_batch_t *b = vb_find(buf, &rx);
    if (b && !rx) {
        /* a DATA frame (its type byte leads the header, src/val_core.c:828-835)
           while batching: the trailer comes later from the window batch;
           control frames (ACK, DONE, ...) go out alone at once, so they are
           computed here */
        if (seed == 0xFFFFFFFFu && len && ((const uint8_t *)buf)[0] == VAL_PKT_DATA && vb_tx_engaged(b) &&
            vb_tx_ready(b)) {
            b->tx_pending = len;
            return 0u;
        }
        return vb_direct(b, seed, buf, len);
    }
    if (b && b->armed && seed == 0xFFFFFFFFu && len == b->armed_len) {
        if (vb_arm_matches(b, (const uint8_t *)buf, len)) {
            b->armed = 0;
            b->st.rx_batched_answers++;
            return b->armed_crc;
        }
        b->st.arm_rejects++;  /* recv_buffer no longer holds the armed frame: computed directly */
    }
    return vb_direct(b, seed, buf, len);
}

/* ---- lifetime ---------------------------------------------------------- */
/* buffers first, so no lookup matches a slot whose batcher is going */
static void vb_release_slot(int i)
{
    __atomic_store_n(&g_buf[0][i], NULL, __ATOMIC_RELEASE);
    __atomic_store_n(&g_buf[1][i], NULL, __ATOMIC_RELEASE);
    __atomic_store_n(&g_reg[i], NULL, __ATOMIC_RELEASE);
}

static void vb_destroy(val_batch_t *b)
{
    vb_free(b->tx, b->tx_pinned);
    vb_free(b->rx, b->rx_pinned);
    free(b->txf);
    free(b->rxf);
    free(b->crc_tmp);
    free(b->off_tmp);
    free(b->len_tmp);
    free(b);
}

val_status_t val_batch_attach(val_config_t *cfg, const val_batch_opts_t *opts, val_batch_t **out)
{
    if (!cfg || !out || !cfg->transport.send || !cfg->transport.recv || !cfg->buffers.send_buffer ||
        !cfg->buffers.recv_buffer || cfg->buffers.packet_size < VAL_WIRE_HEADER_SIZE + VAL_WIRE_TRAILER_SIZE)
        return VAL_ERR_INVALID_ARG;
    /* the provider tells TX from RX by the buffer: they must be distinct, and
       not already attached for another session */
    if (cfg->buffers.send_buffer == cfg->buffers.recv_buffer)
        return VAL_ERR_INVALID_ARG;
    for (int role = 0; role < 2; role++)
        if (vb_lookup(cfg->buffers.send_buffer, role) || vb_lookup(cfg->buffers.recv_buffer, role))
            return VAL_ERR_INVALID_ARG;
    val_batch_t *b = (val_batch_t *)calloc(1, sizeof *b);
    if (!b) return VAL_ERR_NO_MEMORY;
    if (opts) b->opt = *opts;
    else {
        b->opt.tx = VAL_BATCH_AUTO;
        b->opt.rx = VAL_BATCH_AUTO;
    }
    if ((unsigned)b->opt.tx > VAL_BATCH_ALWAYS || (unsigned)b->opt.rx > VAL_BATCH_ALWAYS) {
        free(b);
        return VAL_ERR_INVALID_ARG;
    }
    if (!b->opt.max_frames) b->opt.max_frames = VB_DEFAULT_FRAMES;
    b->mtu = cfg->buffers.packet_size;
    b->win_cap = cfg->tx_flow.window_cap_packets ? cfg->tx_flow.window_cap_packets : 1u;
    if (!b->opt.max_bytes) {  /* the window's bytes, within [16, 256] MiB: a window that can reach the GPU fits */
        const uint64_t w = (uint64_t)b->win_cap * b->mtu;
        b->opt.max_bytes = w < VB_MIN_DEFAULT_BYTES ? VB_MIN_DEFAULT_BYTES
                                                    : w > VB_MAX_DEFAULT_BYTES ? VB_MAX_DEFAULT_BYTES : (size_t)w;
    }
    if (b->opt.max_bytes < b->mtu) b->opt.max_bytes = b->mtu;
    b->cfg = cfg;
    b->u_send = cfg->transport.send;
    b->u_recv = cfg->transport.recv;
    b->u_is_connected = cfg->transport.is_connected;
    b->u_flush = cfg->transport.flush;
    b->u_io = cfg->transport.io_context;
    b->u_provider = cfg->crc32_provider;
    b->ticks = cfg->system.get_ticks_ms;
    b->send_buffer = (const uint8_t *)cfg->buffers.send_buffer;
    b->recv_buffer = (const uint8_t *)cfg->buffers.recv_buffer;
    /* pinned windows (DMA in place on the GPU path) when a device is present;
       a batcher with both directions off never starts the HIP runtime */
    b->pinned = (b->opt.tx || b->opt.rx) && val_gpu_device_count() > 0;
    /* the RX ring holds one frame until RX first batches; the TX window and
       the per-frame arrays come with the first batch (vb_tx_ready,
       vb_rx_ready): a session whose windows never reach the crossover
       allocates no window */
    b->rx_cap = b->mtu;
    b->rx = (uint8_t *)malloc(b->rx_cap);
    int slot = -1;
    for (int i = 0; i < VB_MAX_ATTACHED && slot < 0 && b->rx; i++) {
        val_batch_t *expect = NULL;
        if (__atomic_compare_exchange_n(&g_reg[i], &expect, b, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) slot = i;
    }
    if (!b->rx || slot < 0) {
        const val_status_t st = b->rx ? VAL_ERR_INVALID_ARG : VAL_ERR_NO_MEMORY;
        vb_destroy(b);
        return st;
    }
    __atomic_store_n(&g_buf[0][slot], (const void *)b->send_buffer, __ATOMIC_RELEASE);
    __atomic_store_n(&g_buf[1][slot], (const void *)b->recv_buffer, __ATOMIC_RELEASE);
    int h = __atomic_load_n(&g_hwm, __ATOMIC_ACQUIRE);
    while (h < slot + 1 && !__atomic_compare_exchange_n(&g_hwm, &h, slot + 1, 0, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE)) {
    }
    b->st.status = VAL_OK;
    cfg->transport.send = vb_send;
    cfg->transport.recv = vb_recv;
    cfg->transport.is_connected = b->u_is_connected ? vb_is_connected : NULL;
    cfg->transport.flush = vb_flush_hook;
    cfg->transport.io_context = b;
    cfg->crc32_provider = val_batch_crc32_provider;
    *out = b;
    return VAL_OK;
}

val_status_t val_batch_flush(val_batch_t *b)
{
    return b ? vb_flush_tx(b) : VAL_ERR_INVALID_ARG;
}

void val_batch_get_stats(const val_batch_t *b, val_batch_stats_t *out)
{
    if (!out) return;
    if (!b) {
        memset(out, 0, sizeof *out);
        return;
    }
    *out = b->st;
}

void val_batch_detach(val_batch_t *b)
{
    if (!b) return;
    (void)vb_flush_tx(b);
    for (int i = 0; i < VB_MAX_ATTACHED; i++)
        if (__atomic_load_n(&g_reg[i], __ATOMIC_ACQUIRE) == b) {
            vb_release_slot(i);
            break;
        }
    val_config_t *cfg = b->cfg;
    cfg->transport.send = b->u_send;
    cfg->transport.recv = b->u_recv;
    cfg->transport.is_connected = b->u_is_connected;
    cfg->transport.flush = b->u_flush;
    cfg->transport.io_context = b->u_io;
    cfg->crc32_provider = b->u_provider;
    vb_destroy(b);
}
