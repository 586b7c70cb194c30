/*
 * crc32_oracle.c -- CPU restatement of the reference CRC path.
 * TEST INFRASTRUCTURE ONLY (see crc32_oracle.h): never linked into the product.
 *
 * Follows /root/reference/src/val_core.c:
 *   table generation            :133-148
 *   one-shot val_crc32          :150-160
 *   init/update/finalize state  :162-183
 *   DATA framing + trailer      :718-834 (u16 truncation at :747)
 *   RX trailer compare          :963-974
 * The table is built eagerly and const after that (the reference builds it
 * lazily behind a non-atomic flag, val_core.c:130-148).
 */
#include "crc32_oracle.h"
#include <pthread.h>
#include <string.h>

#define ORACLE_POLY 0xEDB88320u

static uint32_t g_tab[256];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void build_table(void)
{
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int b = 0; b < 8; b++)
            c = (c >> 1) ^ ((c & 1u) ? ORACLE_POLY : 0u);
        g_tab[i] = c;
    }
}

static inline const uint32_t *tab(void)
{
    pthread_once(&g_once, build_table);
    return g_tab;
}

uint32_t oracle_crc32_init_state(void) { return 0xFFFFFFFFu; }

uint32_t oracle_crc32_update_state(uint32_t state, const void *data, size_t len)
{
    const uint32_t *t = tab();
    const uint8_t *p = (const uint8_t *)data;
    for (size_t i = 0; i < len; i++)
        state = t[(state ^ p[i]) & 0xFFu] ^ (state >> 8);
    return state;
}

uint32_t oracle_crc32_finalize_state(uint32_t state) { return state ^ 0xFFFFFFFFu; }

uint32_t oracle_crc32(const void *data, size_t len)
{
    return oracle_crc32_finalize_state(oracle_crc32_update_state(0xFFFFFFFFu, data, len));
}

uint32_t oracle_crc32_provider(uint32_t seed, const void *buf, size_t len)
{
    return oracle_crc32_finalize_state(oracle_crc32_update_state(seed, buf, len));
}

/* ---- GF(2)[x] mod P, reflected representation (bit 31 = x^0) ---------- */
static uint32_t gf_mul(uint32_t a, uint32_t b)
{
    uint32_t prod = 0;
    for (int i = 31; i >= 0; i--) {           /* walk a from x^0 upward */
        if (a & (1u << i))
            prod ^= b;
        b = (b & 1u) ? (b >> 1) ^ ORACLE_POLY : (b >> 1); /* b *= x */
    }
    return prod;
}

/* x^(8n) mod P by square-and-multiply over the bits of n. */
static uint32_t gf_x8n(uint64_t n)
{
    uint32_t result = 0x80000000u;  /* x^0 */
    uint32_t sq = 0x00800000u;      /* x^8 */
    while (n) {
        if (n & 1u)
            result = gf_mul(result, sq);
        sq = gf_mul(sq, sq);
        n >>= 1;
    }
    return result;
}

uint32_t oracle_crc32_shift(uint32_t state, uint64_t nbytes)
{
    return gf_mul(gf_x8n(nbytes), state);
}

uint32_t oracle_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b)
{
    return oracle_crc32_shift(crc_a, len_b) ^ crc_b;
}

/* ---- framing ---------------------------------------------------------- */
static void put_le16(uint8_t *p, uint16_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }
static void put_le32(uint8_t *p, uint32_t v)
{
    for (int i = 0; i < 4; i++) p[i] = (uint8_t)(v >> (8 * i));
}
static void put_le64(uint8_t *p, uint64_t v)
{
    for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i));
}
static uint32_t get_le32(const uint8_t *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

size_t oracle_build_data_frame(const uint8_t *payload, uint32_t payload_len, uint64_t offset,
                               int include_offset, uint8_t *out, size_t out_cap)
{
    uint32_t content_real = payload_len + (include_offset ? 8u : 0u);
    uint16_t content_len = (uint16_t)content_real; /* val_core.c:747 truncation */
    size_t wire = 8u + (size_t)content_len + 4u;
    if (out_cap < wire)
        return 0;
    out[0] = 5u;                                   /* VAL_PKT_DATA */
    out[1] = include_offset ? 1u : 0u;             /* VAL_DATA_OFFSET_PRESENT */
    put_le16(out + 2, content_len);
    put_le32(out + 4, 0u);                         /* type_data = 0 for DATA */
    /* The reference writes the full content into send_buffer but hashes and
     * sends only content_len bytes; emulate what reaches the wire. */
    uint8_t *content = out + 8;
    size_t copied = 0;
    if (include_offset) {
        uint8_t off_le[8];
        put_le64(off_le, offset);
        size_t n = content_len < 8u ? content_len : 8u;
        memcpy(content, off_le, n);
        copied = n;
    }
    if (copied < content_len && payload)
        memcpy(content + copied, payload, content_len - copied);
    uint32_t crc = oracle_crc32(out, 8u + content_len);
    put_le32(out + 8 + content_len, crc);
    return wire;
}

/* ---- batch forms (pthreads, frames round-robin) ----------------------- */
typedef struct {
    const uint8_t *base;
    const uint64_t *off;
    const uint32_t *len;
    uint64_t stride;
    uint32_t flen;
    uint64_t n;
    uint32_t *crc, *hdr;
    uint8_t *ok;
    uint64_t bad;
    int tid, nthreads, mode; /* 0 crc, 1 verify */
} job_t;

static void *worker(void *arg)
{
    job_t *j = (job_t *)arg;
    for (uint64_t i = (uint64_t)j->tid; i < j->n; i += (uint64_t)j->nthreads) {
        const uint8_t *f = j->off ? j->base + j->off[i] : j->base + i * j->stride;
        uint32_t L = j->len ? j->len[i] : j->flen;
        uint32_t c = oracle_crc32(f, L);
        if (j->mode == 0) {
            if (j->crc) j->crc[i] = c;
            if (j->hdr) j->hdr[i] = oracle_crc32(f, L < 8u ? L : 8u);
        } else {
            int good = (c == get_le32(f + L));
            if (j->ok) j->ok[i] = (uint8_t)good;
            j->bad += good ? 0u : 1u;
        }
    }
    return NULL;
}

static uint64_t run_jobs(job_t proto, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    job_t jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = proto;
        jobs[t].tid = t;
        jobs[t].nthreads = nthreads;
        jobs[t].bad = 0;
        if (nthreads == 1) worker(&jobs[t]);
        else pthread_create(&th[t], NULL, worker, &jobs[t]);
    }
    uint64_t bad = 0;
    for (int t = 0; t < nthreads; t++) {
        if (nthreads > 1) pthread_join(th[t], NULL);
        bad += jobs[t].bad;
    }
    return bad;
}

void oracle_crc32_frames(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t n,
                         uint32_t *crc, uint32_t *hdr, int nthreads)
{
    job_t j = {0};
    j.base = base; j.off = off; j.len = len; j.n = n; j.crc = crc; j.hdr = hdr; j.mode = 0;
    run_jobs(j, nthreads);
}

void oracle_crc32_frames_strided(const uint8_t *base, uint64_t stride, uint32_t flen, uint64_t n,
                                 uint32_t *crc, uint32_t *hdr, int nthreads)
{
    job_t j = {0};
    j.base = base; j.stride = stride; j.flen = flen; j.n = n; j.crc = crc; j.hdr = hdr; j.mode = 0;
    run_jobs(j, nthreads);
}

uint64_t oracle_verify_frames(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t n,
                              uint8_t *ok, int nthreads)
{
    job_t j = {0};
    j.base = base; j.off = off; j.len = len; j.n = n; j.ok = ok; j.mode = 1;
    return run_jobs(j, nthreads);
}
