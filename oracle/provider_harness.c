/*
 * provider_harness.c -- drop-in witness (TEST INFRASTRUCTURE).
 *
 * Runs the REFERENCE protocol code (compiled from /root/reference/src into
 * this binary by oracle/Makefile) with the MI355X provider installed exactly
 * the way a VAL user would: cfg.crc32_provider = val_gpu_crc32_provider
 * (reference include/val_protocol.h:264-266). The product library is
 * dlopen'ed RTLD_LOCAL so none of its symbols can interpose on the
 * reference's own val_crc32.
 *
 *   provider_harness <libval_crc_hip.so> tx
 *       DATA frames through val_internal_send_packet_ex (src/val_core.c:874)
 *       with the GPU provider; prints each trailer next to the reference's
 *       own val_crc32 of the same bytes.
 *   provider_harness <libval_crc_hip.so> rx
 *       frames fed to val_internal_recv_packet (src/val_core.c:880) with the
 *       GPU provider: clean frames -> VAL_OK, corrupted -> VAL_ERR_CRC and
 *       metrics.crc_errors++.
 *   provider_harness <libval_crc_hip.so> window <W> <mtu>
 *       a window of W DATA frames framed by the reference
 *       TX path one by one (built-in CRC) vs the batched path of this build
 *       (val_frame_data_batch + one val_crc32_frames_host launch +
 *       val_frame_put_trailers): byte-identical streams required. Then the
 *       stream, with some frames corrupted, goes through the reference RX
 *       (val_internal_recv_packet per frame) and through val_frame_scan +
 *       one val_crc32_verify_frames_host launch: same verdict per frame.
 *   provider_harness <libval_crc_hip.so> windowbench <W> <mtu> <reps>
 *       f1/f2 measured: one window of W DATA frames framed + CRC'd + sent by
 *       the reference TX one frame at a time vs the batched GPU path, and
 *       received + verified by the reference RX vs scan + one GPU verify
 *       (see mode_windowbench).
 *   provider_harness none fixtures
 *       writes tests/golden/dropin_vectors.json (see mode_fixtures): what the
 *       GPU drop-in tests check the product against on the GPU box, where no
 *       reference code exists.
 *   provider_harness none sessions
 *       writes tests/golden/session_vectors.json (see mode_sessions): windowed
 *       and resumed reference sessions, every frame logged.
 *   provider_harness <libval_crc_hip.so|none> loopback <bytes> <mtu> [window]
 *       full val_send_files / val_receive_files transfer over an in-memory
 *       duplex pipe (the reference test strategy), provider on
 *       both sessions ("none" = reference built-in CRC). Prints a digest of
 *       every frame put on the wire so runs can be compared bit for bit, and
 *       how many logged trailers equal the reference's own val_crc32.
 *   provider_harness <libval_crc_hip.so> loopback-batched <bytes> <mtu> <window>
 *       the same transfer with the product's window batcher attached to both
 *       configs (include/val_batch.h: TX trailers from one frames_host call
 *       per window fill, RX frames read ahead and checked from one call).
 *   provider_harness <libval_crc_hip.so> loopback-batched-par <bytes> <mtu> <window> <pairs>
 *       `pairs` batched transfers at once (two threads each): the batcher's
 *       registry and the library under concurrent sessions.
 *   provider_harness <libval_crc_hip.so> sessions | sessions-batched
 *       the five recorded sessions of `none sessions` (windowed, resumed)
 *       re-run with the product's provider installed, plain or batched;
 *       same output format plus the product-side counters.
 * Output: one JSON object per line.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include "prng.h"
#include "val_internal.h"
#include "val_protocol.h"
#include "val_wire.h"

static crc32_func_t g_gpu;
static unsigned long g_calls;
static uint32_t counting_provider(uint32_t seed, const void *buf, size_t len)
{
    __atomic_fetch_add(&g_calls, 1, __ATOMIC_RELAXED);
    return g_gpu(seed, buf, len);
}

static uint32_t ticks(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint32_t)(ts.tv_sec * 1000u + ts.tv_nsec / 1000000u);
}
static void delay(uint32_t ms)
{
    struct timespec ts = {ms / 1000u, (long)(ms % 1000u) * 1000000L};
    nanosleep(&ts, NULL);
}

static uint32_t le32(const uint8_t *p);

/* ---- in-memory byte pipe ------------------------------------------------ */
/* VAL_HARNESS_ZERO_BLOCKS=1: recv with timeout 0 waits until the request can
   be met, as the reference's TCP example does (examples/tcp/common/
   tcp_util.c:383: select with no timeout) */
static int g_zero_blocks;

typedef struct {
    uint8_t *buf;
    size_t cap, head, len;
    pthread_mutex_t mu;
    pthread_cond_t cv;
} pipe_t;

static void pipe_init(pipe_t *p, size_t cap)
{
    p->buf = (uint8_t *)malloc(cap);
    p->cap = cap;
    p->head = p->len = 0;
    pthread_mutex_init(&p->mu, NULL);
    pthread_cond_init(&p->cv, NULL);
}

static void pipe_drain(pipe_t *p)
{
    pthread_mutex_lock(&p->mu);
    p->head = p->len = 0;
    pthread_mutex_unlock(&p->mu);
}

static int pipe_push(pipe_t *p, const uint8_t *d, size_t n)
{
    pthread_mutex_lock(&p->mu);
    if (p->len + n > p->cap) {
        pthread_mutex_unlock(&p->mu);
        return -1;
    }
    const size_t at = (p->head + p->len) % p->cap, first = n < p->cap - at ? n : p->cap - at;
    memcpy(p->buf + at, d, first);  /* the ring's two pieces */
    memcpy(p->buf, d + first, n - first);
    p->len += n;
    pthread_cond_broadcast(&p->cv);
    pthread_mutex_unlock(&p->mu);
    return (int)n;
}

/* Pop exactly n bytes within timeout_ms (0 = nothing, 1 = popped); with
 * upto != 0, pop as soon as any byte is there, at most min(n, upto) of them,
 * and return the count (a transport that delivers partial reads, as the
 * reference's net simulator can: unit_tests/support/test_support.c:655-816). */
static size_t pipe_pop_upto(pipe_t *p, uint8_t *d, size_t n, uint32_t timeout_ms, size_t upto)
{
    struct timespec dl;
    clock_gettime(CLOCK_REALTIME, &dl);
    dl.tv_sec += timeout_ms / 1000u;
    dl.tv_nsec += (long)(timeout_ms % 1000u) * 1000000L;
    if (dl.tv_nsec >= 1000000000L) { dl.tv_sec++; dl.tv_nsec -= 1000000000L; }
    pthread_mutex_lock(&p->mu);
    const size_t need = upto ? 1 : n;
    while (p->len < need) {
        /* timeout 0 is a poll: return at once, as a non-blocking socket does
           (a timed wait on an expired deadline still sleeps ~50-100 us);
           unless told to block, as the reference's TCP example does */
        if (!timeout_ms && g_zero_blocks) {
            pthread_cond_wait(&p->cv, &p->mu);
            continue;
        }
        if (!timeout_ms || pthread_cond_timedwait(&p->cv, &p->mu, &dl) != 0) {
            pthread_mutex_unlock(&p->mu);
            return 0;
        }
    }
    if (upto) {
        n = n < upto ? n : upto;
        n = n < p->len ? n : p->len;
    }
    const size_t first = n < p->cap - p->head ? n : p->cap - p->head;
    memcpy(d, p->buf + p->head, first);
    memcpy(d + first, p->buf, n - first);
    p->head = (p->head + n) % p->cap;
    p->len -= n;
    pthread_mutex_unlock(&p->mu);
    return upto ? n : 1;
}

static int pipe_pop(pipe_t *p, uint8_t *d, size_t n, uint32_t timeout_ms)
{
    struct timespec dl;
    clock_gettime(CLOCK_REALTIME, &dl);
    dl.tv_sec += timeout_ms / 1000u;
    dl.tv_nsec += (long)(timeout_ms % 1000u) * 1000000L;
    if (dl.tv_nsec >= 1000000000L) { dl.tv_sec++; dl.tv_nsec -= 1000000000L; }
    pthread_mutex_lock(&p->mu);
    while (p->len < n) {
        if (!timeout_ms && g_zero_blocks) {
            pthread_cond_wait(&p->cv, &p->mu);
            continue;
        }
        if (!timeout_ms || pthread_cond_timedwait(&p->cv, &p->mu, &dl) != 0) {  /* timeout 0: a poll */
            pthread_mutex_unlock(&p->mu);
            return 0;
        }
    }
    const size_t first = n < p->cap - p->head ? n : p->cap - p->head;
    memcpy(d, p->buf + p->head, first);
    memcpy(d + first, p->buf, n - first);
    p->head = (p->head + n) % p->cap;
    p->len -= n;
    pthread_mutex_unlock(&p->mu);
    return 1;
}

typedef struct {
    uint8_t *bytes;   /* the whole frame as sent */
    size_t len;
    unsigned long epoch;  /* the end's transport.recv calls before this send (sessions mode) */
} frame_rec_t;

typedef struct {
    pipe_t *out, *in;
    uint32_t digest;   /* running CRC (reference val_crc32 state) of all sent bytes */
    unsigned long frames;
    frame_rec_t *log;  /* optional frame log (fixtures mode): one record per transport.send */
    size_t nlog, caplog;
    unsigned long recvs;  /* transport.recv calls of this end: frames sent between two are one window fill */
    unsigned long flip_every, data_sent, flipped;  /* fault injection: one payload bit of every Nth DATA frame */
    uint64_t rng;  /* partial-read sizes (VAL_HARNESS_PARTIAL=rN) */
    unsigned long drop_every, data_sent_d, dropped;  /* fault injection: every Nth DATA frame lost */
    unsigned long fail_at, data_sent_x, send_failures;  /* the fail_at-th DATA frame's send fails, once */
    unsigned long oversize_at, data_sent_o, oversized;  /* the oversize_at-th DATA frame's content_len -> 0xFFFF */
} end_t;

/* VAL_HARNESS_FLIP_EVERY=N: the sender's pipe flips one payload bit of every
 * Nth DATA frame it carries (after logging it), as the reference's own fault
 * injection does (unit_tests/support/test_support.c:488-503); the receiver
 * must count a crc_error for each and the transfer still complete. */
static unsigned long flip_every_env(void)
{
    const char *e = getenv("VAL_HARNESS_FLIP_EVERY");
    return e ? strtoul(e, NULL, 0) : 0ul;
}

/* VAL_HARNESS_DROP_EVERY=N: the sender's pipe loses every Nth DATA frame it
 * carries (after logging it), as the reference's net simulator drops packets
 * (unit_tests/support/test_support.c): the receiver must miss it, the
 * sender retransmit, and the transfer still complete. */
static unsigned long drop_every_env(void)
{
    const char *e = getenv("VAL_HARNESS_DROP_EVERY");
    return e ? strtoul(e, NULL, 0) : 0ul;
}

static int tp_send(void *ctx, const void *data, size_t len)
{
    end_t *e = (end_t *)ctx;
    if (e->fail_at && len > 20 && ((const uint8_t *)data)[0] == VAL_PKT_DATA && ++e->data_sent_x == e->fail_at) {
        e->send_failures++;
        return -1;  /* the transport refused this frame: nothing went on the wire */
    }
    e->digest = val_crc32_update_state(e->digest, data, len);
    e->frames++;
    if (e->caplog) {
        if (e->nlog == e->caplog) {
            e->caplog *= 2;
            e->log = (frame_rec_t *)realloc(e->log, e->caplog * sizeof(frame_rec_t));
        }
        frame_rec_t *r = &e->log[e->nlog++];
        r->bytes = (uint8_t *)malloc(len ? len : 1);
        memcpy(r->bytes, data, len);
        r->len = len;
        r->epoch = e->recvs;
    }
    if (e->drop_every && len > 20 && ((const uint8_t *)data)[0] == VAL_PKT_DATA &&
        ++e->data_sent_d % e->drop_every == 0) {
        e->dropped++;
        return (int)len;  /* "sent": lost on the way */
    }
    if (e->oversize_at && len > 20 && ((const uint8_t *)data)[0] == VAL_PKT_DATA && ++e->data_sent_o == e->oversize_at) {
        /* a header whose content_len exceeds any MTU: the receiver rejects it
           (src/val_core.c:915-921) and reads the rest of the frame as data */
        uint8_t *c = (uint8_t *)malloc(len);
        memcpy(c, data, len);
        c[2] = c[3] = 0xFF;
        e->oversized++;
        const int rc = pipe_push(e->out, c, len);
        free(c);
        return rc;
    }
    if (e->flip_every && len > 20 && ((const uint8_t *)data)[0] == VAL_PKT_DATA &&
        ++e->data_sent % e->flip_every == 0) {
        uint8_t *c = (uint8_t *)malloc(len);
        memcpy(c, data, len);
        c[16 + (e->data_sent * 7u) % (len - 20)] ^= 0x10;  /* a payload byte: header and trailer intact */
        e->flipped++;
        const int rc = pipe_push(e->out, c, len);
        free(c);
        return rc;
    }
    return pipe_push(e->out, (const uint8_t *)data, len);
}

/* VAL_HARNESS_PARTIAL=N: every transport.recv returns at most N bytes (and
 * whatever is there, once anything is): partial reads, which val_recv_full
 * (src/val_core.c:12-43) loops over. */
static size_t g_partial;  /* read once in main, before any session thread */
static int g_coalesce;    /* VAL_HARNESS_COALESCE=1: the batcher's coalesce_send (one send per window) */
/* the batcher's modes (include/val_batch.h: 0 off, 1 auto, 2 always): always by
   default, the mechanics under test; VAL_HARNESS_BATCH=tx|rx|none: one
   direction or neither; VAL_HARNESS_BATCH_MODE=auto: the library's default */
static int g_batch_tx = 2, g_batch_rx = 2;
static uint64_t g_seed;     /* VAL_HARNESS_SEED: partial-read draws */
static int g_partial_random;  /* VAL_HARNESS_PARTIAL=rN: each recv returns 1..N bytes, drawn per call */
static size_t partial_env(void) { return g_partial; }
static size_t partial_draw(end_t *e)
{
    if (!g_partial_random) return g_partial;
    e->rng = e->rng * 6364136223846793005ull + 1442695040888963407ull;  /* per-end LCG: no shared state */
    return 1u + (size_t)((e->rng >> 33) % g_partial);
}

static int tp_recv(void *ctx, void *buffer, size_t size, size_t *got, uint32_t timeout_ms)
{
    end_t *e = (end_t *)ctx;
    e->recvs++;
    if (partial_env()) {
        const size_t n = pipe_pop_upto(e->in, (uint8_t *)buffer, size, timeout_ms, partial_draw(e));
        if (got) *got = n;
        return 0;
    }
    if (pipe_pop(e->in, (uint8_t *)buffer, size, timeout_ms)) {
        if (got) *got = size;
    } else if (got) {
        *got = 0;
    }
    return 0;
}

/* VAL_HARNESS_STALE_ARM=1 (batched loopback): before each of the receiver's
 * frame checks the provider is first called on recv_buffer holding other
 * bytes of the same length (as a resume window read into recv_buffer leaves
 * it, src/val_core.c:431-436) while the batcher has the real frame's CRC
 * armed: the answer must be those bytes' CRC. Then the real call. */
static crc32_func_t g_stale_real;
static const void *g_stale_buf;
static unsigned long g_stale_probes, g_stale_wrong;
static uint32_t stale_probe_provider(uint32_t seed, const void *buf, size_t len)
{
    if (buf == g_stale_buf && seed == 0xFFFFFFFFu && len >= 8) {
        uint8_t *p = (uint8_t *)buf;
        uint8_t *save = (uint8_t *)malloc(len);
        memcpy(save, p, len);
        oracle_prng_fill(0x57A1Eu + g_stale_probes, p, len);
        const uint32_t want = val_crc32(p, len);
        g_stale_wrong += g_stale_real(seed, p, len) != want;
        g_stale_probes++;
        memcpy(p, save, len);
        free(save);
    }
    return g_stale_real(seed, buf, len);
}

static void *fs_open(void *c, const char *path, const char *mode) { (void)c; return fopen(path, mode); }
static size_t fs_read(void *c, void *b, size_t s, size_t n, void *f) { (void)c; return fread(b, s, n, (FILE *)f); }
static size_t fs_write(void *c, const void *b, size_t s, size_t n, void *f) { (void)c; return fwrite(b, s, n, (FILE *)f); }
static int fs_seek(void *c, void *f, int64_t o, int w) { (void)c; return fseeko((FILE *)f, (off_t)o, w); }
static int64_t fs_tell(void *c, void *f) { (void)c; return (int64_t)ftello((FILE *)f); }
static int fs_close(void *c, void *f) { (void)c; return fclose((FILE *)f); }

static void make_cfg(val_config_t *cfg, end_t *e, size_t mtu, crc32_func_t prov)
{
    memset(cfg, 0, sizeof(*cfg));
    cfg->transport.send = tp_send;
    cfg->transport.recv = tp_recv;
    cfg->transport.io_context = e;
    cfg->filesystem.fopen = fs_open;
    cfg->filesystem.fread = fs_read;
    cfg->filesystem.fwrite = fs_write;
    cfg->filesystem.fseek = fs_seek;
    cfg->filesystem.ftell = fs_tell;
    cfg->filesystem.fclose = fs_close;
    cfg->crc32_provider = prov;
    cfg->system.get_ticks_ms = ticks;
    cfg->system.delay_ms = delay;
    cfg->buffers.send_buffer = calloc(1, mtu);
    cfg->buffers.recv_buffer = calloc(1, mtu);
    cfg->buffers.packet_size = mtu;
    cfg->resume.mode = VAL_RESUME_TAIL;
    cfg->resume.tail_cap_bytes = 1024;
    cfg->timeouts.min_timeout_ms = 200;
    cfg->timeouts.max_timeout_ms = 5000;
    /* VAL_HARNESS_MIN_TIMEOUT_MS: a floor that a loaded test host's scheduling
       stalls never reach (runs that compare wire bytes across transports) */
    if (getenv("VAL_HARNESS_MIN_TIMEOUT_MS")) {
        cfg->timeouts.min_timeout_ms = (uint32_t)atoi(getenv("VAL_HARNESS_MIN_TIMEOUT_MS"));
        if (cfg->timeouts.max_timeout_ms < cfg->timeouts.min_timeout_ms) cfg->timeouts.max_timeout_ms = cfg->timeouts.min_timeout_ms;
    }
    /* VAL_HARNESS_MAX_TIMEOUT_MS: a lower ceiling, so a receiver whose peer has
       gone gives up sooner (sendfail) */
    if (getenv("VAL_HARNESS_MAX_TIMEOUT_MS")) {
        const uint32_t m = (uint32_t)atoi(getenv("VAL_HARNESS_MAX_TIMEOUT_MS"));
        cfg->timeouts.max_timeout_ms = m > cfg->timeouts.min_timeout_ms ? m : cfg->timeouts.min_timeout_ms;
    }
    cfg->retries.handshake_retries = 3;
    cfg->retries.meta_retries = 2;
    cfg->retries.data_retries = 4;
    cfg->retries.ack_retries = 6;
    cfg->retries.backoff_ms_base = 10;
}

static void hex(const uint8_t *p, size_t n)
{
    putchar('"');
    for (size_t i = 0; i < n; i++) printf("%02x", p[i]);
    putchar('"');
}

static int mode_tx(void)
{
    const size_t mtu = VAL_MAX_PACKET_SIZE;
    pipe_t a;
    pipe_init(&a, 4u << 20);
    end_t e = {&a, &a, 0xFFFFFFFFu, 0};
    val_config_t cfg;
    make_cfg(&cfg, &e, mtu, counting_provider);
    val_session_t *s = NULL;
    if (val_session_create(&cfg, &s, NULL) != VAL_OK) return 2;
    const uint32_t payloads[] = {0, 1, 3, 492, 1004, 1024, 4093, 16384, 65516, 65527};
    uint8_t *pl = (uint8_t *)malloc(70000), *w = (uint8_t *)malloc(mtu);
    for (size_t i = 0; i < sizeof(payloads) / sizeof(payloads[0]); i++)
        for (int inc = 0; inc <= 1; inc++) {
            oracle_prng_fill(0xF3u ^ ((uint64_t)payloads[i] << 8), pl, payloads[i]);
            size_t before = a.len;
            int rc = val_internal_send_packet_ex(s, VAL_PKT_DATA, pl, payloads[i], (uint64_t)i * 65536u, inc);
            size_t wl = a.len - before;
            pipe_pop(&a, w, wl, 10);
            uint32_t ref = wl >= 12 ? val_crc32(w, wl - 4) : 0u;   /* reference CPU CRC */
            printf("{\"mode\":\"tx\",\"payload_len\":%u,\"include_offset\":%d,\"rc\":%d,\"wire_len\":%zu,\"header\":", payloads[i],
                   inc, rc, wl);
            hex(w, wl >= 8 ? 8 : wl);
            printf(",\"trailer\":");
            hex(w + (wl >= 4 ? wl - 4 : 0), wl >= 4 ? 4 : 0);
            printf(",\"ref_crc\":%u}\n", ref);
        }
    printf("{\"mode\":\"tx_summary\",\"provider_calls\":%lu}\n", g_calls);
    val_session_destroy(s);
    return 0;
}

static int mode_rx(void)
{
    const size_t mtu = 70000;
    pipe_t a;
    pipe_init(&a, 8u << 20);
    end_t e = {&a, &a, 0xFFFFFFFFu, 0};
    val_config_t cfg;
    make_cfg(&cfg, &e, mtu, counting_provider);
    val_session_t *s = NULL;
    if (val_session_create(&cfg, &s, NULL) != VAL_OK) return 2;
    const uint32_t payloads[] = {0, 7, 1004, 16384, 65516};
    uint8_t *pl = (uint8_t *)malloc(70000), *out = (uint8_t *)malloc(70000);
    int idx = 0;
    for (size_t i = 0; i < sizeof(payloads) / sizeof(payloads[0]); i++)
        for (int corrupt = 0; corrupt <= 2; corrupt++) {
            oracle_prng_fill(0xA0u + idx, pl, payloads[i]);
            /* frame it with the reference TX path (reference CRC: provider off) */
            cfg.crc32_provider = NULL;
            val_session_t *txs = NULL;
            val_session_create(&cfg, &txs, NULL);
            size_t before = a.len;
            val_internal_send_packet_ex(txs, VAL_PKT_DATA, pl, payloads[i], 4096u * (uint64_t)idx, 1);
            size_t wl = a.len - before;
            val_session_destroy(txs);
            if (corrupt) {  /* 1: flip a trailer bit, 2: flip a content bit */
                size_t pos = corrupt == 1 ? a.head + before + wl - 1 : a.head + before + 8u + (wl - 12u) / 2u;
                a.buf[pos % a.cap] ^= 0x20;
            }
            uint32_t plen = 0;
            uint64_t off = 0;
            val_packet_type_t t = 0;
            int rc = val_internal_recv_packet(s, &t, out, 70000, &plen, &off, 100);
            val_metrics_t m;
            memset(&m, 0, sizeof m);
            val_get_metrics(s, &m);
            int same = (rc == VAL_OK) ? (plen == payloads[i] && memcmp(out, pl, plen) == 0) : 0;
            printf("{\"mode\":\"rx\",\"payload_len\":%u,\"corrupt\":%d,\"rc\":%d,\"payload_ok\":%d,\"crc_errors\":%u}\n", payloads[i],
                   corrupt, rc, same, m.crc_errors);
            idx++;
        }
    printf("{\"mode\":\"rx_summary\",\"provider_calls\":%lu}\n", g_calls);
    val_session_destroy(s);
    return 0;
}


typedef int (*fn_batch_t)(const uint8_t *, const uint64_t *, const uint32_t *, const uint64_t *, const uint8_t *, uint32_t,
                          uint8_t *, size_t, uint64_t *, uint32_t *, size_t *);
typedef int (*fn_frames_host_t)(const uint8_t *, uint64_t, const uint64_t *, const uint32_t *, uint64_t, uint32_t, uint32_t,
                                uint32_t *, uint32_t *);
typedef void (*fn_put_t)(uint8_t *, const uint64_t *, const uint32_t *, const uint32_t *, uint32_t);
typedef int (*fn_scan_t)(const uint8_t *, size_t, size_t, uint32_t, uint64_t *, uint32_t *, uint32_t *, size_t *);
typedef int (*fn_verify_t)(const uint8_t *, uint64_t, const uint64_t *, const uint32_t *, uint64_t, uint32_t, uint32_t,
                           uint8_t *, uint32_t *);
static void *g_lib;

/* The product's window batcher (include/val_batch.h), reached through dlsym;
 * its two structs restated here because this file compiles against the
 * reference's headers. */
typedef struct {
    uint32_t max_frames;
    size_t max_bytes;
    int tx, rx, coalesce_send, recv_polls;
} hb_opts_t;
typedef struct {
    uint64_t tx_frames, tx_batched_frames, tx_batches, tx_max_batch, rx_frames, rx_batches, rx_max_batch,
        rx_batched_answers, direct_answers, batch_fallbacks;
    int32_t status;
    uint64_t failures, tx_unsent, arm_rejects, resyncs;
} hb_stats_t;
typedef int (*fn_battach_t)(val_config_t *, const hb_opts_t *, void **);
typedef void (*fn_bdetach_t)(void *);
typedef void (*fn_bstats_t)(const void *, hb_stats_t *);
typedef uint64_t (*fn_count_t)(void);

static uint64_t lib_count(const char *name)
{
    fn_count_t f = g_lib ? (fn_count_t)dlsym(g_lib, name) : NULL;
    return f ? f() : 0;
}

/* Attach the batcher to both ends' configs (before val_session_create). */
static int batch_attach(val_config_t *a, val_config_t *b, void **ba, void **bb)
{
    fn_battach_t at = (fn_battach_t)dlsym(g_lib, "val_batch_attach");
    if (!at) return -1;
    /* this harness's recv polls (timeout 0 returns at once) unless told to
       behave like the reference's TCP example (VAL_HARNESS_ZERO_BLOCKS) or
       not to say so (VAL_HARNESS_NO_POLLS) */
    hb_opts_t o = {0, 0, g_batch_tx, g_batch_rx, g_coalesce, !g_zero_blocks && !getenv("VAL_HARNESS_NO_POLLS")};
    if (getenv("VAL_HARNESS_FORCE_POLLS")) o.recv_polls = 1;  /* claim polls even if recv blocks (demonstration) */
    if (getenv("VAL_HARNESS_BATCH_FRAMES")) o.max_frames = (uint32_t)atoi(getenv("VAL_HARNESS_BATCH_FRAMES"));
    if (getenv("VAL_HARNESS_BATCH_BYTES")) o.max_bytes = (size_t)strtoull(getenv("VAL_HARNESS_BATCH_BYTES"), NULL, 0);
    const char *only = getenv("VAL_HARNESS_BATCH_END");  /* sender|receiver: attach one end only */
    if ((!only || strcmp(only, "receiver")) && at(a, &o, ba) != 0) return -1;
    if ((!only || strcmp(only, "sender")) && at(b, &o, bb) != 0) return -1;
    return 0;
}

static void batch_report(FILE *out, void *ba, void *bb)
{
    fn_bstats_t gs = (fn_bstats_t)dlsym(g_lib, "val_batch_get_stats");
    fn_bdetach_t dt = (fn_bdetach_t)dlsym(g_lib, "val_batch_detach");
    hb_stats_t st[2];
    memset(st, 0, sizeof st);
    gs(ba, &st[0]);
    gs(bb, &st[1]);
    fprintf(out, ",\"batch\":[");
    for (int k = 0; k < 2; k++)
        fprintf(out, "%s{\"end\":\"%s\",\"tx_frames\":%llu,\"tx_batched_frames\":%llu,\"tx_batches\":%llu,\"tx_max_batch\":%llu,"
               "\"rx_frames\":%llu,\"rx_batches\":%llu,\"rx_max_batch\":%llu,\"rx_batched_answers\":%llu,"
               "\"direct_answers\":%llu,\"batch_fallbacks\":%llu,\"status\":%d,\"failures\":%llu,\"tx_unsent\":%llu,"
               "\"arm_rejects\":%llu,\"resyncs\":%llu}",
               k ? "," : "", k ? "receiver" : "sender", (unsigned long long)st[k].tx_frames,
               (unsigned long long)st[k].tx_batched_frames, (unsigned long long)st[k].tx_batches,
               (unsigned long long)st[k].tx_max_batch, (unsigned long long)st[k].rx_frames,
               (unsigned long long)st[k].rx_batches, (unsigned long long)st[k].rx_max_batch,
               (unsigned long long)st[k].rx_batched_answers, (unsigned long long)st[k].direct_answers,
               (unsigned long long)st[k].batch_fallbacks, st[k].status, (unsigned long long)st[k].failures,
               (unsigned long long)st[k].tx_unsent, (unsigned long long)st[k].arm_rejects,
               (unsigned long long)st[k].resyncs);
    fprintf(out, "]");
    dt(ba);
    dt(bb);
}

static int mode_window(uint32_t W, size_t mtu)
{
    fn_batch_t batch = (fn_batch_t)dlsym(g_lib, "val_frame_data_batch");
    fn_frames_host_t frames = (fn_frames_host_t)dlsym(g_lib, "val_crc32_frames_host");
    fn_put_t put = (fn_put_t)dlsym(g_lib, "val_frame_put_trailers");
    fn_scan_t scan = (fn_scan_t)dlsym(g_lib, "val_frame_scan");
    fn_verify_t verify = (fn_verify_t)dlsym(g_lib, "val_crc32_verify_frames_host");
    if (!batch || !frames || !put || !scan || !verify) return 2;
    /* The sender's window: max payload MTU-12, minus 8 with an explicit offset
       (src/val_sender.c:271-277); offset explicit on the first frame of the
       window (include_offset = next_to_send == last_acked, :833). */
    const size_t maxp = mtu - 12;
    const uint64_t file_size = (uint64_t)W * maxp - 777u;
    uint8_t *file = (uint8_t *)malloc(file_size);
    oracle_prng_fill(0x3171D0, file, file_size);
    uint64_t *pay_off = calloc(W, 8), *file_off = calloc(W, 8), *fo = calloc(W, 8), *fo2 = calloc(W, 8);
    uint32_t *pay_len = calloc(W, 4), *cl = calloc(W, 4), *cl2 = calloc(W, 4), *crc = calloc(W, 4);
    uint8_t *inc = calloc(W, 1), *ok = calloc(W, 1);
    uint32_t nf = 0;
    for (uint64_t pos = 0; pos < file_size && nf < W; nf++) {
        inc[nf] = (nf % 5 == 0);
        size_t take = maxp - (inc[nf] ? 8u : 0u);
        if (take > file_size - pos) take = (size_t)(file_size - pos);
        pay_off[nf] = pos;
        file_off[nf] = pos;
        pay_len[nf] = (uint32_t)take;
        pos += take;
    }
    /* reference TX, one frame at a time */
    pipe_t a;
    pipe_init(&a, (size_t)W * mtu + 4096);
    end_t e = {&a, &a, 0xFFFFFFFFu, 0};
    val_config_t cfg;
    make_cfg(&cfg, &e, mtu, NULL);
    val_session_t *s = NULL;
    if (val_session_create(&cfg, &s, NULL) != VAL_OK) return 3;
    for (uint32_t i = 0; i < nf; i++)
        if (val_internal_send_packet_ex(s, VAL_PKT_DATA, file + pay_off[i], pay_len[i], file_off[i], inc[i]) != VAL_OK) return 4;
    const size_t ref_len = a.len;
    uint8_t *ref = (uint8_t *)malloc(ref_len);
    pipe_pop(&a, ref, ref_len, 10);
    /* batched TX on the GPU */
    uint8_t *stage = (uint8_t *)malloc((size_t)W * mtu);
    size_t used = 0;
    int st = batch(file, pay_off, pay_len, file_off, inc, nf, stage, (size_t)W * mtu, fo, cl, &used);
    if (st != 0) return 5;
    st = frames(stage, used, fo, cl, 0, 0, nf, crc, NULL);
    if (st != 0) return 6;
    put(stage, fo, cl, crc, nf);
    const int tx_equal = (used == ref_len) && memcmp(stage, ref, ref_len) == 0;
    /* corrupt some frames of the reference stream, then verify both ways */
    uint32_t corrupted = 0;
    for (uint32_t i = 3; i < nf; i += 7) {
        ref[fo[i] + 8u + (i * 13u) % (cl[i] - 8u)] ^= (uint8_t)(1u << (i % 8));
        corrupted++;
    }
    uint32_t nscan = 0;
    size_t consumed = 0;
    st = scan(ref, ref_len, mtu, nf, fo2, cl2, &nscan, &consumed);
    uint32_t nbad = 0;
    int vst = verify(ref, ref_len, fo2, cl2, 0, 0, nscan, ok, &nbad);
    pipe_push(&a, ref, ref_len);
    val_config_t rcfg;
    make_cfg(&rcfg, &e, mtu, NULL);
    val_session_t *r = NULL;
    if (val_session_create(&rcfg, &r, NULL) != VAL_OK) return 7;
    uint8_t *out = (uint8_t *)malloc(mtu);
    uint32_t same_verdict = 0, ref_bad = 0;
    for (uint32_t i = 0; i < nf; i++) {
        val_packet_type_t t = 0;
        uint32_t plen = 0;
        uint64_t off = 0;
        int rc = val_internal_recv_packet(r, &t, out, (uint32_t)mtu, &plen, &off, 100);
        ref_bad += (rc == VAL_ERR_CRC);
        same_verdict += ((rc == VAL_OK) == (i < nscan && ok[i] == 1));
    }
    val_metrics_t m;
    memset(&m, 0, sizeof m);
    val_get_metrics(r, &m);
    printf("{\"mode\":\"window\",\"frames\":%u,\"mtu\":%zu,\"wire_bytes\":%zu,\"tx_equal\":%d,\"scan_status\":%d,\"scanned\":%u,"
           "\"consumed\":%zu,\"verify_status\":%d,\"gpu_bad\":%u,\"ref_bad\":%u,\"ref_crc_errors\":%u,\"corrupted\":%u,"
           "\"same_verdict\":%u}\n",
           nf, mtu, ref_len, tx_equal, st, nscan, consumed, vst, nbad, ref_bad, m.crc_errors, corrupted, same_verdict);
    val_session_destroy(s);
    val_session_destroy(r);
    return 0;
}

/* ---- windowbench: call-site batching measured end to end
 * Linear in-memory transport (memcpy; no digest), so the timed work is the
 * framing + CRC + transport copy of one window of W DATA frames:
 *   ref_tx   reference TX, one val_internal_send_packet_ex per frame (CPU CRC)
 *   gpu_tx   val_frame_data_batch into a pinned window buffer + one
 *            val_crc32_frames_host launch + val_frame_put_trailers + one
 *            transport send per frame
 *   ref_rx   reference RX, one val_internal_recv_packet per frame (CPU CRC)
 *   gpu_rx   the window's bytes read in one transport call into a pinned
 *            ring + val_frame_scan + one val_crc32_verify_frames_host launch
 * Median of REPS windows each; parity: byte-identical TX streams, every frame
 * accepted on both RX paths. */
typedef struct {
    uint8_t *buf;
    size_t cap, wpos, rpos;
} sink_t;

static int sink_send(void *ctx, const void *data, size_t len)
{
    sink_t *k = (sink_t *)ctx;
    if (k->wpos + len > k->cap) return -1;
    memcpy(k->buf + k->wpos, data, len);
    k->wpos += len;
    return (int)len;
}

static int sink_recv(void *ctx, void *buffer, size_t size, size_t *got, uint32_t timeout_ms)
{
    (void)timeout_ms;
    sink_t *k = (sink_t *)ctx;
    const size_t n = size <= k->wpos - k->rpos ? size : k->wpos - k->rpos;
    memcpy(buffer, k->buf + k->rpos, n);
    k->rpos += n;
    if (got) *got = n;
    return 0;
}

static double now_us(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e6 + ts.tv_nsec / 1e3;
}

static int cmp_d(const void *a, const void *b)
{
    const double x = *(const double *)a, y = *(const double *)b;
    return (x > y) - (x < y);
}

static double median(double *v, int n)
{
    qsort(v, (size_t)n, sizeof(double), cmp_d);
    return v[n / 2];
}

typedef void *(*fn_alloc_t)(size_t);

static int mode_windowbench(uint32_t W, size_t mtu, int reps)
{
    fn_batch_t batch = (fn_batch_t)dlsym(g_lib, "val_frame_data_batch");
    fn_frames_host_t frames = (fn_frames_host_t)dlsym(g_lib, "val_crc32_frames_host");
    fn_put_t put = (fn_put_t)dlsym(g_lib, "val_frame_put_trailers");
    fn_scan_t scan = (fn_scan_t)dlsym(g_lib, "val_frame_scan");
    fn_verify_t verify = (fn_verify_t)dlsym(g_lib, "val_crc32_verify_frames_host");
    fn_alloc_t halloc = (fn_alloc_t)dlsym(g_lib, "val_gpu_host_alloc");
    if (!batch || !frames || !put || !scan || !verify || !halloc) return 2;
    const size_t maxp = mtu - 12;
    const uint64_t file_size = (uint64_t)W * (maxp - 8);
    uint8_t *file = (uint8_t *)malloc(file_size);
    oracle_prng_fill(0x5151, file, file_size);
    uint64_t *pay_off = calloc(W, 8), *file_off = calloc(W, 8), *fo = calloc(W, 8), *fo2 = calloc(W, 8);
    uint32_t *pay_len = calloc(W, 4), *cl = calloc(W, 4), *cl2 = calloc(W, 4), *crc = calloc(W, 4);
    uint8_t *inc = calloc(W, 1), *ok = calloc(W, 1);
    uint32_t nf = 0;
    for (uint64_t pos = 0; pos < file_size && nf < W; nf++) {
        inc[nf] = (nf == 0); /* explicit offset on the window's first frame (src/val_sender.c:833) */
        size_t take = maxp - (inc[nf] ? 8u : 0u);
        if (take > file_size - pos) take = (size_t)(file_size - pos);
        pay_off[nf] = file_off[nf] = pos;
        pay_len[nf] = (uint32_t)take;
        pos += take;
    }
    const size_t cap = (size_t)W * mtu + 4096;
    sink_t ks = {(uint8_t *)malloc(cap), cap, 0, 0};
    val_config_t cfg;
    make_cfg(&cfg, NULL, mtu, NULL);
    cfg.transport.send = sink_send;
    cfg.transport.recv = sink_recv;
    cfg.transport.io_context = &ks;
    val_session_t *s = NULL;
    if (val_session_create(&cfg, &s, NULL) != VAL_OK) return 3;
    double *t = (double *)malloc(sizeof(double) * (size_t)reps);
    /* reference TX */
    for (int r = 0; r < reps; r++) {
        ks.wpos = 0;
        const double t0 = now_us();
        for (uint32_t i = 0; i < nf; i++)
            if (val_internal_send_packet_ex(s, VAL_PKT_DATA, file + pay_off[i], pay_len[i], file_off[i], inc[i]) != VAL_OK) return 4;
        t[r] = now_us() - t0;
    }
    const double ref_tx = median(t, reps);
    const size_t wire = ks.wpos;
    uint8_t *ref = (uint8_t *)malloc(wire);
    memcpy(ref, ks.buf, wire);
    /* batched GPU TX */
    uint8_t *stage = (uint8_t *)halloc((size_t)W * mtu);
    if (!stage) return 5;
    size_t used = 0;
    for (int r = 0; r < reps; r++) {
        ks.wpos = 0;
        const double t0 = now_us();
        if (batch(file, pay_off, pay_len, file_off, inc, nf, stage, (size_t)W * mtu, fo, cl, &used) != 0) return 6;
        if (frames(stage, used, fo, cl, 0, 0, nf, crc, NULL) != 0) return 7;
        put(stage, fo, cl, crc, nf);
        for (uint32_t i = 0; i < nf; i++) sink_send(&ks, stage + fo[i], cl[i] + 4u);
        t[r] = now_us() - t0;
    }
    const double gpu_tx = median(t, reps);
    const int tx_equal = ks.wpos == wire && memcmp(ks.buf, ref, wire) == 0;
    /* reference RX */
    uint8_t *out = (uint8_t *)malloc(mtu);
    uint32_t ref_ok = 0;
    for (int r = 0; r < reps; r++) {
        ks.rpos = 0;
        uint32_t good = 0;
        const double t0 = now_us();
        for (uint32_t i = 0; i < nf; i++) {
            val_packet_type_t ty = 0;
            uint32_t plen = 0;
            uint64_t off = 0;
            good += val_internal_recv_packet(s, &ty, out, (uint32_t)mtu, &plen, &off, 100) == VAL_OK;
        }
        t[r] = now_us() - t0;
        ref_ok = good;
    }
    const double ref_rx = median(t, reps);
    /* batched GPU RX */
    uint8_t *ring = (uint8_t *)halloc(wire);
    if (!ring) return 8;
    uint32_t nscan = 0, nbad = 0;
    int vst = 0;
    for (int r = 0; r < reps; r++) {
        ks.rpos = 0;
        const double t0 = now_us();
        size_t got = 0, consumed = 0;
        sink_recv(&ks, ring, wire, &got, 0);
        if (scan(ring, got, mtu, nf, fo2, cl2, &nscan, &consumed) != 0) return 9;
        vst = verify(ring, got, fo2, cl2, 0, 0, nscan, ok, &nbad);
        t[r] = now_us() - t0;
    }
    const double gpu_rx = median(t, reps);
    printf("{\"mode\":\"windowbench\",\"frames\":%u,\"mtu\":%zu,\"wire_bytes\":%zu,\"reps\":%d,"
           "\"ref_tx_us\":%.1f,\"gpu_tx_us\":%.1f,\"ref_rx_us\":%.1f,\"gpu_rx_us\":%.1f,"
           "\"tx_equal\":%d,\"ref_rx_ok\":%u,\"gpu_rx_scanned\":%u,\"gpu_rx_status\":%d,\"gpu_rx_bad\":%u}\n",
           nf, mtu, wire, reps, ref_tx, gpu_tx, ref_rx, gpu_rx, tx_equal, ref_ok, nscan, vst, nbad);
    val_session_destroy(s);
    return 0;
}

typedef struct {
    val_session_t *rx;
    const char *dir;
    val_status_t st;
} rx_job_t;

static void *rx_main(void *arg)
{
    rx_job_t *j = (rx_job_t *)arg;
    j->st = val_receive_files(j->rx, j->dir);
    return NULL;
}

/* Every frame an end put on the wire carries the reference's own CRC
 * (val_crc32 of this binary) as its trailer: counted over the frame log. A
 * logged send may hold several frames back to back (the batcher's
 * coalesce_send): they are split by their headers' content_len. */
static unsigned long trailers_ok_n(const end_t *e, unsigned long *frames)
{
    unsigned long n = 0, k = 0;
    for (size_t i = 0; i < e->nlog; i++) {
        const uint8_t *f = e->log[i].bytes;
        const size_t wl = e->log[i].len;
        for (size_t pos = 0; pos + 12 <= wl;) {
            const size_t fl = 12u + (size_t)(f[pos + 2] | f[pos + 3] << 8);
            const size_t use = fl <= wl - pos ? fl : wl - pos;
            n += val_crc32(f + pos, use - 4) == le32(f + pos + use - 4);
            k++;
            pos += use;
        }
    }
    if (frames) *frames = k;
    return n;
}
static unsigned long trailers_ok(const end_t *e) { return trailers_ok_n(e, NULL); }

static int loopback_run(FILE *out_json, size_t bytes, size_t mtu, int use_gpu, uint16_t window, int batched,
                        uint64_t seed)
{
    char tmpl[] = "/tmp/valgpuXXXXXX";
    char *dir = mkdtemp(tmpl);
    if (!dir) return 2;
    char in[512], outdir[512], out[512];
    snprintf(in, sizeof in, "%s/input.bin", dir);
    snprintf(outdir, sizeof outdir, "%s/out", dir);
    snprintf(out, sizeof out, "%s/out/input.bin", dir);
    mkdir(outdir, 0777);
    uint8_t *data = (uint8_t *)malloc(bytes ? bytes : 1);
    oracle_prng_fill(seed, data, bytes);
    FILE *f = fopen(in, "wb");
    fwrite(data, 1, bytes, f);
    fclose(f);

    pipe_t a2b, b2a;
    /* room for two full windows in flight (64 MiB at least) */
    const size_t pwin = (size_t)2u * (window ? window : 1u) * mtu + ((size_t)1u << 20);
    const size_t pcap = pwin > ((size_t)64u << 20) ? pwin : ((size_t)64u << 20);
    pipe_init(&a2b, pcap);
    pipe_init(&b2a, pcap);
    end_t etx = {&a2b, &b2a, 0xFFFFFFFFu, 0, NULL, 0, 0, 0}, erx = {&b2a, &a2b, 0xFFFFFFFFu, 0, NULL, 0, 0, 0};
    etx.caplog = erx.caplog = 4096;
    etx.log = (frame_rec_t *)malloc(etx.caplog * sizeof(frame_rec_t));
    erx.log = (frame_rec_t *)malloc(erx.caplog * sizeof(frame_rec_t));
    etx.flip_every = flip_every_env();
    etx.drop_every = drop_every_env();
    etx.oversize_at = getenv("VAL_HARNESS_OVERSIZE_AT") ? strtoul(getenv("VAL_HARNESS_OVERSIZE_AT"), NULL, 0) : 0ul;
    etx.rng = g_seed * 2u + 1u;  /* partial-read draws (VAL_HARNESS_PARTIAL=rN), per end */
    erx.rng = g_seed * 2u + 2u;
    crc32_func_t prov = use_gpu ? counting_provider : NULL;
    val_config_t ctx_, crx;
    make_cfg(&ctx_, &etx, mtu, prov);
    make_cfg(&crx, &erx, mtu, prov);
    if (window) {
        ctx_.tx_flow.window_cap_packets = crx.tx_flow.window_cap_packets = window;
        ctx_.tx_flow.initial_cwnd_packets = crx.tx_flow.initial_cwnd_packets = window;
    }
    void *ba = NULL, *bb = NULL;
    const uint64_t cpu_b0 = lib_count("val_gpu_cpu_batch_count"), cpu_s0 = lib_count("val_gpu_cpu_small_count"),
                   cpu_f0 = lib_count("val_gpu_cpu_fallback_count");
    if (batched && batch_attach(&ctx_, &crx, &ba, &bb) != 0) return 4;
    const int stale = batched && getenv("VAL_HARNESS_STALE_ARM") && atoi(getenv("VAL_HARNESS_STALE_ARM"));
    if (stale) {  /* the receiver's provider, wrapped before its session copies the config */
        g_stale_real = crx.crc32_provider;
        g_stale_buf = crx.buffers.recv_buffer;
        crx.crc32_provider = stale_probe_provider;
    }
    val_session_t *tx = NULL, *rx = NULL;
    if (val_session_create(&ctx_, &tx, NULL) != VAL_OK || val_session_create(&crx, &rx, NULL) != VAL_OK) return 3;
    rx_job_t job = {rx, outdir, VAL_OK};
    pthread_t th;
    pthread_create(&th, NULL, rx_main, &job);
    const char *files[1] = {in};
    uint32_t t0 = ticks();
    val_status_t st = val_send_files(tx, files, 1, NULL);
    pthread_join(th, NULL);
    uint32_t t1 = ticks();
    val_metrics_t mt, mr;
    memset(&mt, 0, sizeof mt);
    memset(&mr, 0, sizeof mr);
    val_get_metrics(tx, &mt);
    val_get_metrics(rx, &mr);
    int equal = 0;
    unsigned long wf_tx = 0, wf_rx = 0;
    const unsigned long t_ok = trailers_ok_n(&etx, &wf_tx) + trailers_ok_n(&erx, &wf_rx);
    FILE *g = fopen(out, "rb");
    if (g) {
        uint8_t *back = (uint8_t *)malloc(bytes + 1);
        size_t r = fread(back, 1, bytes + 1, g);
        fclose(g);
        equal = (r == bytes) && memcmp(back, data, bytes) == 0;
        free(back);
    }
    fprintf(out_json, "{\"mode\":\"loopback\",\"gpu\":%d,\"batched\":%d,\"window\":%u,\"bytes\":%zu,\"mtu\":%zu,\"tx_status\":%d,"
           "\"rx_status\":%d,\"equal\":%d,"
           "\"tx_crc_errors\":%u,\"rx_crc_errors\":%u,\"retransmits\":%u,\"timeouts\":%u,\"tx_frames\":%lu,\"rx_frames\":%lu,"
           "\"tx_digest\":%u,\"rx_digest\":%u,\"trailers_ok\":%lu,\"wire_frames\":%lu,\"flipped\":%lu,\"dropped\":%lu,\"oversized\":%lu,\"provider_calls\":%lu,\"wall_ms\":%u,"
           "\"lib_cpu_batches\":%llu,\"lib_cpu_small\":%llu,\"lib_cpu_fallbacks\":%llu,\"stale_probes\":%lu,"
           "\"stale_wrong\":%lu",
           use_gpu, batched, window, bytes, mtu, st, job.st, equal, mt.crc_errors, mr.crc_errors, mt.retransmits + mr.retransmits,
           mt.timeouts + mr.timeouts, etx.frames, erx.frames, etx.digest ^ 0xFFFFFFFFu, erx.digest ^ 0xFFFFFFFFu,
           t_ok, wf_tx + wf_rx, etx.flipped, etx.dropped, etx.oversized, __atomic_load_n(&g_calls, __ATOMIC_RELAXED), t1 - t0,
           (unsigned long long)(lib_count("val_gpu_cpu_batch_count") - cpu_b0),
           (unsigned long long)(lib_count("val_gpu_cpu_small_count") - cpu_s0),
           (unsigned long long)(lib_count("val_gpu_cpu_fallback_count") - cpu_f0), stale ? g_stale_probes : 0ul,
           stale ? g_stale_wrong : 0ul);
    val_session_destroy(tx);
    val_session_destroy(rx);
    if (stale) crx.crc32_provider = g_stale_real;  /* detach restores what attach saw */
    if (batched) batch_report(out_json, ba, bb);
    fprintf(out_json, "}\n");
    for (size_t i = 0; i < etx.nlog; i++) free(etx.log[i].bytes);
    for (size_t i = 0; i < erx.nlog; i++) free(erx.log[i].bytes);
    free(etx.log);
    free(erx.log);
    free(data);
    remove(out);
    remove(in);
    rmdir(outdir);
    rmdir(dir);
    return 0;
}

/* provider_harness <lib|none> sendfail|oversize <bytes> <mtu> <window> <k> [batched]
 * Two transfers on one pair of sessions; a fault in the first, the second
 * clean. sendfail: the sender's transport fails the k-th DATA frame's send
 * (once); in the reference val_send_files returns VAL_ERR_IO at that frame
 * (src/val_core.c:835-842, src/val_sender.c:835-840) and the receiver's
 * transfer ends on its own timeouts. oversize: the k-th DATA frame arrives
 * with content_len 0xFFFF; the receiver rejects it (src/val_core.c:915-921)
 * and, in the reference, that transfer fails. The second transfer resumes the
 * receiver's partial file (VAL_RESUME_TAIL). Prints both transfers'
 * statuses, the sender's last error detail, its wire digest and frames at
 * the end of the first, and whether the second transfer's file arrived
 * whole. */
static int mode_twice(size_t bytes, size_t mtu, int use_gpu, uint16_t window, int oversize, unsigned long k, int batched)
{
    char tmpl[] = "/tmp/valfailXXXXXX";
    char *dir = mkdtemp(tmpl);
    if (!dir) return 2;
    char in[512], outdir[512], out[512];
    snprintf(in, sizeof in, "%s/input.bin", dir);
    snprintf(outdir, sizeof outdir, "%s/out", dir);
    snprintf(out, sizeof out, "%s/out/input.bin", dir);
    mkdir(outdir, 0777);
    uint8_t *data = (uint8_t *)malloc(bytes ? bytes : 1);
    oracle_prng_fill(0xFA11u, data, bytes);
    FILE *f = fopen(in, "wb");
    fwrite(data, 1, bytes, f);
    fclose(f);
    pipe_t a2b, b2a;
    const size_t pwin = (size_t)2u * (window ? window : 1u) * mtu + ((size_t)1u << 20);
    const size_t pcap = pwin > ((size_t)64u << 20) ? pwin : ((size_t)64u << 20);
    pipe_init(&a2b, pcap);
    pipe_init(&b2a, pcap);
    end_t etx, erx;
    memset(&etx, 0, sizeof etx);
    memset(&erx, 0, sizeof erx);
    etx.out = &a2b;
    etx.in = &b2a;
    erx.out = &b2a;
    erx.in = &a2b;
    etx.digest = erx.digest = 0xFFFFFFFFu;
    if (oversize) etx.oversize_at = k;
    else etx.fail_at = k;
    val_config_t ctx_, crx;
    make_cfg(&ctx_, &etx, mtu, use_gpu ? counting_provider : NULL);
    make_cfg(&crx, &erx, mtu, use_gpu ? counting_provider : NULL);
    if (window) {
        ctx_.tx_flow.window_cap_packets = crx.tx_flow.window_cap_packets = window;
        ctx_.tx_flow.initial_cwnd_packets = crx.tx_flow.initial_cwnd_packets = window;
    }
    void *ba = NULL, *bb = NULL;
    if (batched && batch_attach(&ctx_, &crx, &ba, &bb) != 0) return 4;
    val_session_t *tx = NULL, *rx = NULL;
    if (val_session_create(&ctx_, &tx, NULL) != VAL_OK || val_session_create(&crx, &rx, NULL) != VAL_OK) return 3;
    const char *files[1] = {in};
    val_status_t st[2], rst[2], code = VAL_OK;
    uint32_t detail = 0;
    uint32_t digest1 = 0;
    unsigned long frames1 = 0;
    for (int t = 0; t < 2; t++) {
        rx_job_t job = {rx, outdir, VAL_OK};
        pthread_t th;
        pthread_create(&th, NULL, rx_main, &job);
        st[t] = val_send_files(tx, files, 1, NULL);
        if (t == 0) {
            val_get_last_error(tx, &code, &detail);
            digest1 = etx.digest ^ 0xFFFFFFFFu;
            frames1 = etx.frames;
            etx.fail_at = etx.oversize_at = 0;  /* the second transfer runs clean */
        }
        pthread_join(th, NULL);
        rst[t] = job.st;
        if (t == 0 && oversize) {
            /* after a protocol error the application reconnects: the old
               connection's bytes are gone (both directions) */
            pipe_drain(&a2b);
            pipe_drain(&b2a);
        }
    }
    int equal = 0;
    FILE *g = fopen(out, "rb");
    if (g) {
        uint8_t *back = (uint8_t *)malloc(bytes + 1);
        size_t r = fread(back, 1, bytes + 1, g);
        fclose(g);
        equal = (r == bytes) && memcmp(back, data, bytes) == 0;
        free(back);
    }
    printf("{\"mode\":\"%s\",\"gpu\":%d,\"batched\":%d,\"window\":%u,\"bytes\":%zu,\"mtu\":%zu,\"fail_at\":%lu,"
           "\"tx_status1\":%d,\"rx_status1\":%d,\"tx_error1\":%d,\"tx_detail1\":%u,\"tx_digest1\":%u,\"tx_frames1\":%lu,"
           "\"send_failures\":%lu,\"tx_status2\":%d,\"rx_status2\":%d,\"equal2\":%d",
           oversize ? "oversize" : "sendfail", use_gpu, batched, window, bytes, mtu, k, st[0], rst[0], code, detail, digest1, frames1, etx.send_failures, st[1],
           rst[1], equal);
    val_session_destroy(tx);
    val_session_destroy(rx);
    if (batched) batch_report(stdout, ba, bb);
    printf("}\n");
    free(data);
    remove(out);
    remove(in);
    rmdir(outdir);
    rmdir(dir);
    return 0;
}

static int mode_loopback(size_t bytes, size_t mtu, int use_gpu, uint16_t window, int batched)
{
    return loopback_run(stdout, bytes, mtu, use_gpu, window, batched, 0x10AD);
}

/* `pairs` batched loopback transfers at once, one sender and one receiver
 * thread each: every session's provider calls and window batches go through
 * the one process-wide batcher registry and the product library at the same
 * time (reference include/val_protocol.h:231-233: sessions run in parallel). */
typedef struct {
    size_t bytes, mtu;
    uint16_t window;
    uint64_t seed;
    char *buf;
    size_t len;
    int rc;
} par_job_t;

static void *par_main(void *arg)
{
    par_job_t *j = (par_job_t *)arg;
    FILE *m = open_memstream(&j->buf, &j->len);
    j->rc = loopback_run(m, j->bytes, j->mtu, 1, j->window, 1, j->seed);
    fclose(m);
    return NULL;
}

static int mode_loopback_par(size_t bytes, size_t mtu, uint16_t window, int pairs)
{
    par_job_t *jobs = (par_job_t *)calloc((size_t)pairs, sizeof(par_job_t));
    pthread_t *th = (pthread_t *)calloc((size_t)pairs, sizeof(pthread_t));
    const uint64_t cpu_b0 = lib_count("val_gpu_cpu_batch_count"), cpu_s0 = lib_count("val_gpu_cpu_small_count"),
                   cpu_f0 = lib_count("val_gpu_cpu_fallback_count");
    for (int i = 0; i < pairs; i++) {
        jobs[i] = (par_job_t){bytes, mtu, window, 0x10AD + 977u * (uint64_t)i, NULL, 0, 0};
        pthread_create(&th[i], NULL, par_main, &jobs[i]);
    }
    int rc = 0;
    printf("{\"mode\":\"loopback-batched-par\",\"pairs\":%d,\"lib_cpu_batches\":", pairs);
    for (int i = 0; i < pairs; i++) pthread_join(th[i], NULL);
    printf("%llu,\"lib_cpu_small\":%llu,\"lib_cpu_fallbacks\":%llu,\"runs\":[",
           (unsigned long long)(lib_count("val_gpu_cpu_batch_count") - cpu_b0),
           (unsigned long long)(lib_count("val_gpu_cpu_small_count") - cpu_s0),
           (unsigned long long)(lib_count("val_gpu_cpu_fallback_count") - cpu_f0));
    for (int i = 0; i < pairs; i++) {
        size_t n = jobs[i].len;
        while (n && (jobs[i].buf[n - 1] == '\n')) n--;
        printf("%s%.*s", i ? "," : "", (int)n, jobs[i].buf);
        rc |= jobs[i].rc;
        free(jobs[i].buf);
    }
    printf("]}\n");
    free(jobs);
    free(th);
    return rc;
}

/* ---- fixtures: drop-in golden vectors, reference built-in CRC only --------
 * `provider_harness none fixtures > tests/golden/dropin_vectors.json`.
 * Everything the GPU drop-in tests need to check the product against the
 * reference without running reference code on the GPU box: TX frames of
 * val_internal_send_packet_ex, RX verdicts of val_internal_recv_packet on
 * clean and corrupted frames, TX windows of W frames with corrupted-frame
 * verdicts, and the F6 frame log of the 1 MiB / MTU 1024
 * loopback transfer (BASELINE configs[0]). Payload bytes are not stored: they
 * are oracle_prng_fill streams the tests regenerate (tests/_prng.py). */
static void fx_hex(const uint8_t *p, size_t n) { hex(p, n); }

static uint32_t le32(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
static uint64_t le64(const uint8_t *p) { return (uint64_t)le32(p) | (uint64_t)le32(p + 4) << 32; }

static void fx_tx(void)
{
    const size_t mtu = VAL_MAX_PACKET_SIZE;
    pipe_t a;
    pipe_init(&a, 4u << 20);
    end_t e = {&a, &a, 0xFFFFFFFFu, 0};
    val_config_t cfg;
    make_cfg(&cfg, &e, mtu, NULL);
    val_session_t *s = NULL;
    val_session_create(&cfg, &s, NULL);
    const uint32_t payloads[] = {0, 1, 3, 492, 1004, 1024, 4093, 16384, 65516, 65527, 65528, 65536};
    uint8_t *pl = (uint8_t *)malloc(70000), *w = (uint8_t *)malloc(mtu);
    printf("\"tx\":[");
    int first = 1;
    for (size_t i = 0; i < sizeof(payloads) / sizeof(payloads[0]); i++)
        for (int inc = 0; inc <= 1; inc++) {
            const uint64_t seed = 0xF3u ^ ((uint64_t)payloads[i] << 8);
            const uint64_t off = (uint64_t)i * 65536u + (inc ? (1ull << 32) + 5u : 0u);
            oracle_prng_fill(seed, pl, payloads[i]);
            size_t before = a.len;
            int rc = val_internal_send_packet_ex(s, VAL_PKT_DATA, pl, payloads[i], off, inc);
            size_t wl = a.len - before;
            pipe_pop(&a, w, wl, 10);
            printf("%s\n{\"payload_len\":%u,\"include_offset\":%d,\"offset\":%llu,\"seed\":%llu,\"rc\":%d,\"wire_len\":%zu,"
                   "\"prefix\":",
                   first ? "" : ",", payloads[i], inc, (unsigned long long)off, (unsigned long long)seed, rc, wl);
            fx_hex(w, wl >= 4 ? (wl - 4 < 16 ? wl - 4 : 16) : 0);
            printf(",\"trailer\":%u}", wl >= 4 ? le32(w + wl - 4) : 0u);
            first = 0;
        }
    printf("],\n");
    val_session_destroy(s);
    free(pl);
    free(w);
}

static void fx_rx(void)
{
    const size_t mtu = 70000;
    pipe_t a;
    pipe_init(&a, 8u << 20);
    end_t e = {&a, &a, 0xFFFFFFFFu, 0};
    val_config_t cfg;
    make_cfg(&cfg, &e, mtu, NULL);
    val_session_t *s = NULL;
    val_session_create(&cfg, &s, NULL);
    const uint32_t payloads[] = {0, 7, 1004, 16384, 65516};
    uint8_t *pl = (uint8_t *)malloc(70000), *out = (uint8_t *)malloc(70000);
    int idx = 0;
    printf("\"rx\":[");
    for (size_t i = 0; i < sizeof(payloads) / sizeof(payloads[0]); i++)
        for (int corrupt = 0; corrupt <= 3; corrupt++) {
            const uint64_t seed = 0xA0u + (uint64_t)idx;
            oracle_prng_fill(seed, pl, payloads[i]);
            val_session_t *txs = NULL;
            val_session_create(&cfg, &txs, NULL);
            size_t before = a.len;
            val_internal_send_packet_ex(txs, VAL_PKT_DATA, pl, payloads[i], 4096u * (uint64_t)idx, 1);
            size_t wl = a.len - before;
            val_session_destroy(txs);
            const uint32_t trailer = (uint32_t)a.buf[(a.head + before + wl - 4) % a.cap] |
                                     (uint32_t)a.buf[(a.head + before + wl - 3) % a.cap] << 8 |
                                     (uint32_t)a.buf[(a.head + before + wl - 2) % a.cap] << 16 |
                                     (uint32_t)a.buf[(a.head + before + wl - 1) % a.cap] << 24;
            /* 1: trailer bit, 2: content bit, 3: header (content_len kept, type_data bit) */
            size_t pos = 0;
            const uint8_t mask = 0x20;
            if (corrupt) {
                pos = corrupt == 1 ? wl - 1 : corrupt == 2 ? 8u + (wl - 12u) / 2u : 5u;
                a.buf[(a.head + before + pos) % a.cap] ^= mask;
            }
            uint32_t plen = 0;
            uint64_t off = 0;
            val_packet_type_t t = 0;
            int rc = val_internal_recv_packet(s, &t, out, 70000, &plen, &off, 100);
            val_metrics_t m;
            memset(&m, 0, sizeof m);
            val_get_metrics(s, &m);
            int same = (rc == VAL_OK) ? (plen == payloads[i] && memcmp(out, pl, plen) == 0) : 0;
            printf("%s\n{\"payload_len\":%u,\"seed\":%llu,\"offset\":%llu,\"trailer\":%u,\"corrupt\":%d,\"pos\":%zu,\"mask\":%u,"
                   "\"rc\":%d,\"payload_ok\":%d,\"crc_errors\":%u}",
                   idx ? "," : "", payloads[i], (unsigned long long)seed, 4096ull * (unsigned long long)idx, trailer, corrupt,
                   pos, corrupt ? mask : 0u, rc, same, m.crc_errors);
            idx++;
        }
    printf("],\n");
    val_session_destroy(s);
    free(pl);
    free(out);
}

/* One TX window of W frames (sender layout, src/val_sender.c:271-277,833), as
 * mode_window, reference only. */
static void fx_window(uint32_t W, size_t mtu, int last)
{
    const size_t maxp = mtu - 12;
    const uint64_t file_size = (uint64_t)W * maxp - 777u;
    const uint64_t file_seed = 0x3171D0;
    uint8_t *file = (uint8_t *)malloc(file_size);
    oracle_prng_fill(file_seed, file, file_size);
    uint64_t *pay_off = calloc(W, 8);
    uint32_t *pay_len = calloc(W, 4);
    uint8_t *inc = calloc(W, 1);
    uint32_t nf = 0;
    for (uint64_t pos = 0; pos < file_size && nf < W; nf++) {
        inc[nf] = (nf % 5 == 0);
        size_t take = maxp - (inc[nf] ? 8u : 0u);
        if (take > file_size - pos) take = (size_t)(file_size - pos);
        pay_off[nf] = pos;
        pay_len[nf] = (uint32_t)take;
        pos += take;
    }
    pipe_t a;
    pipe_init(&a, (size_t)W * mtu + 4096);
    end_t e = {&a, &a, 0xFFFFFFFFu, 0};
    val_config_t cfg;
    make_cfg(&cfg, &e, mtu, NULL);
    val_session_t *s = NULL;
    val_session_create(&cfg, &s, NULL);
    for (uint32_t i = 0; i < nf; i++) val_internal_send_packet_ex(s, VAL_PKT_DATA, file + pay_off[i], pay_len[i], pay_off[i], inc[i]);
    const size_t ref_len = a.len;
    uint8_t *ref = (uint8_t *)malloc(ref_len);
    pipe_pop(&a, ref, ref_len, 10);
    printf("{\"W\":%u,\"mtu\":%zu,\"file_seed\":%llu,\"file_size\":%llu,\"frames\":[", W, mtu, (unsigned long long)file_seed,
           (unsigned long long)file_size);
    for (uint32_t i = 0; i < nf; i++)
        printf("%s[%llu,%u,%u]", i ? "," : "", (unsigned long long)pay_off[i], pay_len[i], inc[i]);
    /* frame offsets in the stream from the headers; trailers; stream digest */
    uint64_t *fo = calloc(nf, 8);
    uint32_t *cl = calloc(nf, 4);
    size_t p = 0;
    printf("],\"trailers\":[");
    for (uint32_t i = 0; i < nf; i++) {
        fo[i] = p;
        cl[i] = 8u + ((uint32_t)ref[p + 2] | (uint32_t)ref[p + 3] << 8);
        printf("%s%u", i ? "," : "", le32(ref + p + cl[i]));
        p += cl[i] + 4u;
    }
    printf("],\"wire_bytes\":%zu,\"wire_crc\":%u,\"corrupt\":[", ref_len, val_crc32(ref, ref_len));
    int firstc = 1;
    for (uint32_t i = 3; i < nf; i += 7) {
        const size_t pos = fo[i] + 8u + (i * 13u) % (cl[i] - 8u);
        const uint8_t mask = (uint8_t)(1u << (i % 8));
        ref[pos] ^= mask;
        printf("%s[%u,%zu,%u]", firstc ? "" : ",", i, pos, mask);
        firstc = 0;
    }
    pipe_push(&a, ref, ref_len);
    val_config_t rcfg;
    make_cfg(&rcfg, &e, mtu, NULL);
    val_session_t *r = NULL;
    val_session_create(&rcfg, &r, NULL);
    uint8_t *out = (uint8_t *)malloc(mtu);
    printf("],\"ref_rc\":[");
    for (uint32_t i = 0; i < nf; i++) {
        val_packet_type_t t = 0;
        uint32_t plen = 0;
        uint64_t off = 0;
        int rc = val_internal_recv_packet(r, &t, out, (uint32_t)mtu, &plen, &off, 100);
        printf("%s%d", i ? "," : "", rc);
    }
    val_metrics_t m;
    memset(&m, 0, sizeof m);
    val_get_metrics(r, &m);
    printf("],\"ref_crc_errors\":%u}%s\n", m.crc_errors, last ? "" : ",");
    val_session_destroy(s);
    val_session_destroy(r);
    free(file);
    free(ref);
    free(out);
    free(fo);
    free(cl);
    free(pay_off);
    free(pay_len);
    free(inc);
}

/* F6: the frame log of both sessions' transport.send during a 1 MiB / MTU
 * 1024 loopback (reference harness unit_tests/send_receive/test_single_file.c:
 * 9-11,155-161). Per frame: [type, wire_len, trailer, file_off, prefix_hex]:
 * DATA frames (type 5) carry the first 8 (implied offset) or 16 bytes and the
 * file offset of their payload (-1 otherwise); other frames carry every byte
 * but the trailer. */
static void fx_log(const end_t *e, const uint8_t *file, size_t bytes)
{
    uint64_t next = 0;
    for (size_t i = 0; i < e->nlog; i++) {
        const uint8_t *f = e->log[i].bytes;
        const size_t wl = e->log[i].len;
        const uint32_t content = (uint32_t)f[2] | (uint32_t)f[3] << 8;
        long long foff = -1;
        size_t pre = wl - 4;
        if (f[0] == VAL_PKT_DATA) {
            const int explicit_off = f[1] & 1u;
            const uint64_t off = explicit_off ? le64(f + 8) : next;
            const uint32_t plen = content - (explicit_off ? 8u : 0u);
            const uint8_t *pay = f + 8 + (explicit_off ? 8 : 0);
            if (off + plen > bytes || memcmp(pay, file + off, plen) != 0) {
                fprintf(stderr, "fixtures: DATA frame %zu payload is not file[%llu:+%u]\n", i, (unsigned long long)off, plen);
                exit(3);
            }
            foff = (long long)off;
            next = off + plen;
            pre = explicit_off ? 16 : 8;
        }
        printf("%s\n[%u,%zu,%u,%lld,", i ? "," : "", f[0], wl, le32(f + wl - 4), foff);
        fx_hex(f, pre);
        putchar(']');
    }
}

static int mode_fixtures(void)
{
    printf("{\"generator\":\"oracle/provider_harness none fixtures (reference src/ built by oracle/Makefile, built-in CRC)\",\n");
    fx_tx();
    fx_rx();
    printf("\"windows\":[\n");
    fx_window(64, 1024, 0);
    fx_window(33, 16404, 0);
    fx_window(16, 65536, 0);
    fx_window(7, 512, 0);
    fx_window(300, 1024, 1);
    printf("],\n");
    /* F6 loopback, reference CRC on both sessions */
    const size_t bytes = 1048576, mtu = 1024;
    char tmpl[] = "/tmp/valfxXXXXXX";
    char *dir = mkdtemp(tmpl);
    if (!dir) return 2;
    /* relative paths: the META frame carries the sender path, so the log
       must not depend on the temporary directory's name */
    char cwd[1024];
    if (!getcwd(cwd, sizeof cwd) || chdir(dir) != 0) return 2;
    const char *in = "input.bin", *outdir = "out", *out = "out/input.bin";
    mkdir(outdir, 0777);
    uint8_t *data = (uint8_t *)malloc(bytes);
    oracle_prng_fill(0x10AD, data, bytes);
    FILE *f = fopen(in, "wb");
    fwrite(data, 1, bytes, f);
    fclose(f);
    pipe_t a2b, b2a;
    pipe_init(&a2b, 64u << 20);
    pipe_init(&b2a, 64u << 20);
    end_t etx = {&a2b, &b2a, 0xFFFFFFFFu, 0, NULL, 0, 0}, erx = {&b2a, &a2b, 0xFFFFFFFFu, 0, NULL, 0, 0};
    etx.caplog = erx.caplog = 4096;
    etx.log = (frame_rec_t *)malloc(etx.caplog * sizeof(frame_rec_t));
    erx.log = (frame_rec_t *)malloc(erx.caplog * sizeof(frame_rec_t));
    val_config_t ctx_, crx;
    make_cfg(&ctx_, &etx, mtu, NULL);
    make_cfg(&crx, &erx, mtu, NULL);
    val_session_t *tx = NULL, *rx = NULL;
    if (val_session_create(&ctx_, &tx, NULL) != VAL_OK || val_session_create(&crx, &rx, NULL) != VAL_OK) return 3;
    rx_job_t job = {rx, outdir, VAL_OK};
    pthread_t th;
    pthread_create(&th, NULL, rx_main, &job);
    const char *files[1] = {in};
    val_status_t st = val_send_files(tx, files, 1, NULL);
    pthread_join(th, NULL);
    val_metrics_t mt, mr;
    memset(&mt, 0, sizeof mt);
    memset(&mr, 0, sizeof mr);
    val_get_metrics(tx, &mt);
    val_get_metrics(rx, &mr);
    int equal = 0;
    FILE *g = fopen(out, "rb");
    if (g) {
        uint8_t *back = (uint8_t *)malloc(bytes + 1);
        size_t r = fread(back, 1, bytes + 1, g);
        fclose(g);
        equal = (r == bytes) && memcmp(back, data, bytes) == 0;
        free(back);
    }
    if (st != VAL_OK || job.st != VAL_OK || !equal || mt.retransmits + mr.retransmits || mt.timeouts + mr.timeouts) {
        fprintf(stderr, "fixtures: loopback not clean (tx %d rx %d equal %d)\n", st, job.st, equal);
        return 4;
    }
    printf("\"loopback\":{\"bytes\":%zu,\"mtu\":%zu,\"file_seed\":%d,\"tx_crc_errors\":%u,\"rx_crc_errors\":%u,"
           "\"file_crc\":%u,\"tx_digest\":%u,\"rx_digest\":%u,\"tx_frames\":[",
           bytes, mtu, 0x10AD, mt.crc_errors, mr.crc_errors, val_crc32(data, bytes), etx.digest ^ 0xFFFFFFFFu,
           erx.digest ^ 0xFFFFFFFFu);
    fx_log(&etx, data, bytes);
    printf("],\"rx_frames\":[");
    fx_log(&erx, data, bytes);
    printf("]}}\n");
    val_session_destroy(tx);
    val_session_destroy(rx);
    remove(out);
    remove(in);
    rmdir(outdir);
    if (chdir(cwd) != 0) return 5;
    rmdir(dir);
    return 0;
}

/* ---- sessions: real reference sessions for the call-site fixtures ---------
 * `provider_harness none sessions > tests/golden/session_vectors.json`.
 * Full val_send_files / val_receive_files transfers (reference built-in CRC)
 * whose every transport.send is logged as in F6, plus each frame's window
 * epoch: the number of transport.recv calls its end had made before the send,
 * so frames sent back to back without a receive are one window fill of the
 * sender (src/val_sender.c:822-841; include_offset = next_to_send ==
 * last_acked, :833, visible as flags bit 0 of each DATA frame).
 *   windowed loopbacks: tx_flow.window_cap_packets = 64 on both ends
 *       (negotiation src/val_core.c:1755,1810-1834), initial window 64, at
 *       MTU 1,024 and 16,404;
 *   resumed VAL_RESUME_TAIL transfers: the receiver's output file already
 *       holds a prefix of the input, so the receiver sends its tail-window
 *       CRC in RESUME_RESP (src/val_receiver.c:158-181), the sender computes
 *       the same window over its file and sends a VERIFY request
 *       (src/val_sender.c:205-252), and the receiver checks it
 *       (src/val_receiver.c:431-444): at the default 8 MiB cap, at 1 KiB,
 *       and once with a byte of the receiver's tail flipped (verify fails).
 * The wire is timing dependent (ACKs race the window fill), so this file is
 * a recording, not a regenerable golden: tests check it for internal
 * consistency on the CPU and replay it through the product on the GPU. */
static void fx_log_epochs(const end_t *e, const uint8_t *file, size_t bytes)
{
    uint64_t next = 0;
    for (size_t i = 0; i < e->nlog; i++) {
        const uint8_t *f = e->log[i].bytes;
        const size_t wl = e->log[i].len;
        const uint32_t content = (uint32_t)f[2] | (uint32_t)f[3] << 8;
        long long foff = -1;
        size_t pre = wl - 4;
        if (f[0] == VAL_PKT_DATA) {
            const int explicit_off = f[1] & 1u;
            const uint64_t off = explicit_off ? le64(f + 8) : next;
            const uint32_t plen = content - (explicit_off ? 8u : 0u);
            const uint8_t *pay = f + 8 + (explicit_off ? 8 : 0);
            if (off + plen > bytes || memcmp(pay, file + off, plen) != 0) {
                fprintf(stderr, "sessions: DATA frame %zu payload is not file[%llu:+%u]\n", i, (unsigned long long)off, plen);
                exit(3);
            }
            foff = (long long)off;
            next = off + plen;
            pre = explicit_off ? 16 : 8;
        }
        printf("%s\n[%u,%zu,%u,%lld,", i ? "," : "", f[0], wl, le32(f + wl - 4), foff);
        fx_hex(f, pre);
        printf(",%lu]", e->log[i].epoch);
    }
}

/* One session: `bytes` of input (oracle_prng_fill(seed)); when existing > 0
 * the receiver's output file starts as the input's first `existing` bytes
 * (byte `flip` XOR 0x5A when flip >= 0). */
static int fx_session(const char *name, size_t bytes, size_t mtu, uint16_t window, uint32_t tail_cap, size_t existing,
                      long long flip, uint64_t seed, int last, crc32_func_t prov, int batched)
{
    char tmpl[] = "/tmp/valssXXXXXX";
    char *dir = mkdtemp(tmpl);
    if (!dir) return 2;
    char cwd[1024];
    if (!getcwd(cwd, sizeof cwd) || chdir(dir) != 0) return 2;
    const char *in = "input.bin", *outdir = "out", *out = "out/input.bin";
    mkdir(outdir, 0777);
    uint8_t *data = (uint8_t *)malloc(bytes);
    oracle_prng_fill(seed, data, bytes);
    FILE *f = fopen(in, "wb");
    fwrite(data, 1, bytes, f);
    fclose(f);
    if (existing) {
        uint8_t *part = (uint8_t *)malloc(existing);
        memcpy(part, data, existing);
        if (flip >= 0) part[flip] ^= 0x5A;
        FILE *g = fopen(out, "wb");
        fwrite(part, 1, existing, g);
        fclose(g);
        free(part);
    }
    pipe_t a2b, b2a;
    pipe_init(&a2b, 64u << 20);
    pipe_init(&b2a, 64u << 20);
    end_t etx = {&a2b, &b2a, 0xFFFFFFFFu, 0, NULL, 0, 0, 0}, erx = {&b2a, &a2b, 0xFFFFFFFFu, 0, NULL, 0, 0, 0};
    etx.caplog = erx.caplog = 4096;
    etx.log = (frame_rec_t *)malloc(etx.caplog * sizeof(frame_rec_t));
    erx.log = (frame_rec_t *)malloc(erx.caplog * sizeof(frame_rec_t));
    val_config_t ctx_, crx;
    make_cfg(&ctx_, &etx, mtu, prov);
    make_cfg(&crx, &erx, mtu, prov);
    ctx_.tx_flow.window_cap_packets = crx.tx_flow.window_cap_packets = window;
    ctx_.tx_flow.initial_cwnd_packets = crx.tx_flow.initial_cwnd_packets = window;
    ctx_.resume.tail_cap_bytes = crx.resume.tail_cap_bytes = tail_cap;
    void *ba = NULL, *bb = NULL;
    const uint64_t cpu_b0 = lib_count("val_gpu_cpu_batch_count"), cpu_s0 = lib_count("val_gpu_cpu_small_count"),
                   cpu_f0 = lib_count("val_gpu_cpu_fallback_count");
    if (batched && batch_attach(&ctx_, &crx, &ba, &bb) != 0) return 4;
    val_session_t *tx = NULL, *rx = NULL;
    if (val_session_create(&ctx_, &tx, NULL) != VAL_OK || val_session_create(&crx, &rx, NULL) != VAL_OK) return 3;
    rx_job_t job = {rx, outdir, VAL_OK};
    pthread_t th;
    pthread_create(&th, NULL, rx_main, &job);
    const char *files[1] = {in};
    val_status_t st = val_send_files(tx, files, 1, NULL);
    pthread_join(th, NULL);
    val_metrics_t mt, mr;
    memset(&mt, 0, sizeof mt);
    memset(&mr, 0, sizeof mr);
    val_get_metrics(tx, &mt);
    val_get_metrics(rx, &mr);
    int equal = 0;
    FILE *g = fopen(out, "rb");
    if (g) {
        uint8_t *back = (uint8_t *)malloc(bytes + 1);
        size_t r = fread(back, 1, bytes + 1, g);
        fclose(g);
        equal = (r == bytes) && memcmp(back, data, bytes) == 0;
        free(back);
    }
    printf("{\"name\":\"%s\",\"bytes\":%zu,\"mtu\":%zu,\"window_cap_packets\":%u,\"tail_cap_bytes\":%u,\"existing\":%zu,"
           "\"flip\":%lld,\"file_seed\":%llu,\"tx_status\":%d,\"rx_status\":%d,\"equal\":%d,\"tx_crc_errors\":%u,"
           "\"rx_crc_errors\":%u,\"retransmits\":%u,\"file_crc\":%u,\"tx_frames\":[",
           name, bytes, mtu, window, tail_cap, existing, flip, (unsigned long long)seed, st, job.st, equal, mt.crc_errors,
           mr.crc_errors, mt.retransmits + mr.retransmits, val_crc32(data, bytes));
    fx_log_epochs(&etx, data, bytes);
    printf("],\"rx_frames\":[");
    fx_log_epochs(&erx, data, bytes);
    printf("]");
    if (prov) {  /* the product installed: every logged trailer against the reference's own val_crc32 */
        printf(",\"provider\":\"%s\",\"trailers_ok\":%lu,\"frames_logged\":%zu,\"lib_cpu_batches\":%llu,"
               "\"lib_cpu_small\":%llu,\"lib_cpu_fallbacks\":%llu",
               batched ? "batched" : "product", trailers_ok(&etx) + trailers_ok(&erx), etx.nlog + erx.nlog,
               (unsigned long long)(lib_count("val_gpu_cpu_batch_count") - cpu_b0),
               (unsigned long long)(lib_count("val_gpu_cpu_small_count") - cpu_s0),
               (unsigned long long)(lib_count("val_gpu_cpu_fallback_count") - cpu_f0));
    }
    val_session_destroy(tx);
    val_session_destroy(rx);
    if (batched) batch_report(stdout, ba, bb);
    printf("}%s\n", last ? "" : ",");
    for (size_t i = 0; i < etx.nlog; i++) free(etx.log[i].bytes);
    for (size_t i = 0; i < erx.nlog; i++) free(erx.log[i].bytes);
    free(etx.log);
    free(erx.log);
    free(data);
    remove(out);
    remove(in);
    rmdir(outdir);
    if (chdir(cwd) != 0) return 5;
    rmdir(dir);
    return 0;
}

/* prov NULL: the reference's built-in CRC (the recorded fixtures); else the
 * product's provider installed on both ends, optionally with the batcher. */
static int mode_sessions(crc32_func_t prov, int batched)
{
    int rc = 0;
    printf("{\"generator\":\"oracle/provider_harness %s sessions (reference src/ built by oracle/Makefile, %s)\",\n"
           "\"sessions\":[\n", prov ? "<lib>" : "none",
           prov ? (batched ? "product provider + val_batch window batching" : "product provider") : "built-in CRC");
    rc |= fx_session("window64_mtu1024", 600000, 1024, 64, 1024, 0, -1, 0x5E55101, 0, prov, batched);
    rc |= fx_session("window64_mtu16404", 3u << 20, 16404, 64, 1024, 0, -1, 0x5E55102, 0, prov, batched);
    rc |= fx_session("resume_tail_cap8m", (12u << 20) + 777u, 4096, 16, 0, (10u << 20) + 12345u, -1, 0x5E55103, 0, prov,
                     batched);
    rc |= fx_session("resume_tail_cap1k", 400000, 1024, 8, 1024, 300005, -1, 0x5E55104, 0, prov, batched);
    rc |= fx_session("resume_tail_mismatch", 400000, 1024, 8, 8192, 300005, 300005 - 100, 0x5E55105, 1, prov, batched);
    printf("]}\n");
    return rc;
}

int main(int argc, char **argv)
{
    const char *pe = getenv("VAL_HARNESS_PARTIAL");
    g_partial_random = pe && pe[0] == 'r';
    g_seed = getenv("VAL_HARNESS_SEED") ? strtoull(getenv("VAL_HARNESS_SEED"), NULL, 0) : 0u;
    g_partial = pe ? (size_t)strtoul(pe + g_partial_random, NULL, 0) : 0;
    g_zero_blocks = getenv("VAL_HARNESS_ZERO_BLOCKS") && atoi(getenv("VAL_HARNESS_ZERO_BLOCKS"));
    const char *ce = getenv("VAL_HARNESS_COALESCE");
    g_coalesce = ce ? atoi(ce) : 0;
    const char *be = getenv("VAL_HARNESS_BATCH");
    if (be && !strcmp(be, "tx")) g_batch_rx = 0;
    if (be && !strcmp(be, "rx")) g_batch_tx = 0;
    if (be && !strcmp(be, "none")) g_batch_tx = g_batch_rx = 0;
    const char *bm = getenv("VAL_HARNESS_BATCH_MODE");
    if (bm && !strcmp(bm, "auto")) {
        g_batch_tx = g_batch_tx ? 1 : 0;
        g_batch_rx = g_batch_rx ? 1 : 0;
    }
    (void)val_crc32_init_state();  /* the reference's lazy table (src/val_core.c:133-148), before any thread */
    if (argc >= 3 && !strcmp(argv[1], "none") && !strcmp(argv[2], "fixtures")) return mode_fixtures();
    if (argc >= 3 && !strcmp(argv[1], "none") && !strcmp(argv[2], "sessions")) return mode_sessions(NULL, 0);
    if (argc < 3) {
        fprintf(stderr, "usage: %s <libval_crc_hip.so|none> tx|rx|loopback [bytes mtu]\n", argv[0]);
        return 1;
    }
    int use_gpu = strcmp(argv[1], "none") != 0;
    if (use_gpu) {
        void *h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
        g_lib = h;
        if (!h) {
            fprintf(stderr, "dlopen: %s\n", dlerror());
            return 1;
        }
        g_gpu = (crc32_func_t)dlsym(h, "val_gpu_crc32_provider");
        int (*init)(int) = (int (*)(int))dlsym(h, "val_gpu_init");
        if (!g_gpu || !init) {
            fprintf(stderr, "GPU provider unavailable\n");
            return 1;
        }
        /* Without a device the product still answers below its thresholds
           (its CPU engine); the tx/rx/window modes need the GPU. */
        const int have_gpu = init(0) == 0;
        if (!have_gpu && (!strcmp(argv[2], "tx") || !strcmp(argv[2], "rx") || !strncmp(argv[2], "window", 6))) {
            fprintf(stderr, "no HIP device\n");
            return 1;
        }
        (void)g_gpu(0xFFFFFFFFu, "warm", 4); /* first call pays HIP init, not the protocol */
        g_calls = 0;
    }
    if (!strcmp(argv[2], "tx")) return use_gpu ? mode_tx() : 1;
    if (!strcmp(argv[2], "rx")) return use_gpu ? mode_rx() : 1;
    if (!strcmp(argv[2], "window") && argc >= 5)
        return use_gpu ? mode_window((uint32_t)strtoul(argv[3], NULL, 0), (size_t)strtoull(argv[4], NULL, 0)) : 1;
    if (!strcmp(argv[2], "windowbench") && argc >= 6)
        return use_gpu ? mode_windowbench((uint32_t)strtoul(argv[3], NULL, 0), (size_t)strtoull(argv[4], NULL, 0),
                                          atoi(argv[5]))
                       : 1;
    if (!strcmp(argv[2], "loopback") && argc >= 5)
        return mode_loopback((size_t)strtoull(argv[3], NULL, 0), (size_t)strtoull(argv[4], NULL, 0), use_gpu,
                             argc >= 6 ? (uint16_t)strtoul(argv[5], NULL, 0) : 0, 0);
    if (!strcmp(argv[2], "loopback-batched") && argc >= 6)
        return use_gpu ? mode_loopback((size_t)strtoull(argv[3], NULL, 0), (size_t)strtoull(argv[4], NULL, 0), 1,
                                       (uint16_t)strtoul(argv[5], NULL, 0), 1)
                       : 1;
    if (!strcmp(argv[2], "loopback-batched-par") && argc >= 7)
        return use_gpu ? mode_loopback_par((size_t)strtoull(argv[3], NULL, 0), (size_t)strtoull(argv[4], NULL, 0),
                                           (uint16_t)strtoul(argv[5], NULL, 0), atoi(argv[6]))
                       : 1;
    if ((!strcmp(argv[2], "sendfail") || !strcmp(argv[2], "oversize")) && argc >= 7)
        return mode_twice((size_t)strtoull(argv[3], NULL, 0), (size_t)strtoull(argv[4], NULL, 0), use_gpu,
                          (uint16_t)strtoul(argv[5], NULL, 0), !strcmp(argv[2], "oversize"), strtoul(argv[6], NULL, 0),
                          argc >= 8 && use_gpu ? atoi(argv[7]) : 0);
    if (!strcmp(argv[2], "sessions")) return use_gpu ? mode_sessions(counting_provider, 0) : 1;
    if (!strcmp(argv[2], "sessions-batched")) return use_gpu ? mode_sessions(counting_provider, 1) : 1;
    fprintf(stderr, "bad mode\n");
    return 1;
}
