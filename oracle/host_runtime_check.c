/* Host-runtime check (TEST INFRASTRUCTURE, CPU only): the library's host
 * paths that run without a GPU -- the CPU engine behind val_crc32_frames_host
 * and its helper threads, verify with corrupted trailers and payload states,
 * the *_host_multi CPU route, the region CPU route, the scalar hooks -- driven
 * from several threads at once with random batches, every output against
 * this oracle. Built with a sanitizer by tools/sanitize_host_runtime.sh.
 * usage: host_runtime_check THREADS ITERS SEED ; prints one JSON line, exit 1
 * on any mismatch. */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "crc32_oracle.h"
#include "prng.h"
#include "val_crc32_gpu.h"
#include "val_wire.h"

static int g_iters;
static uint64_t g_seed;
static unsigned long g_bad, g_checked;
static pthread_mutex_t g_mu = PTHREAD_MUTEX_INITIALIZER;

static void bad(const char *what, unsigned t, int it, uint64_t i)
{
    pthread_mutex_lock(&g_mu);
    if (g_bad < 20) fprintf(stderr, "BAD %s thread %u iter %d item %llu\n", what, t, it, (unsigned long long)i);
    g_bad++;
    pthread_mutex_unlock(&g_mu);
}

static uint32_t le32(const uint8_t *p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }

static void *worker(void *arg)
{
    const unsigned t = (unsigned)(uintptr_t)arg;
    unsigned long checked = 0;
    for (int it = 0; it < g_iters; it++) {
        const uint64_t r = oracle_splitmix64(g_seed + t * 7919u, (uint64_t)it);
        /* a packed, unaligned stream of n frames of CRC input len[i] + 4-byte
           trailer; total from a few KiB to ~24 MiB (the helper-thread path
           starts at 8 MiB with 2+ threads) */
        const uint32_t n = 1u + (uint32_t)(r % 3000u);
        const uint32_t maxlen = (it % 4 == 3) ? 16400u : 1u + (uint32_t)((r >> 16) % 4000u);
        uint64_t *off = malloc(n * sizeof *off);
        uint32_t *len = malloc(n * sizeof *len), *crc = malloc(n * 4u), *hdr = malloc(n * 4u), *pay = malloc(n * 4u);
        uint8_t *ok = malloc(n);
        uint64_t total = 0, pos = (r >> 40) & 15u;
        for (uint32_t i = 0; i < n; i++) {
            len[i] = (uint32_t)(oracle_splitmix64(r, i) % maxlen);
            off[i] = pos;
            pos += len[i] + 4u;
            total += len[i];
        }
        const uint64_t base_len = pos;
        uint8_t *base = malloc(base_len ? base_len : 1);
        oracle_prng_fill(r ^ 0xABCDEFu, base, base_len);
        for (uint32_t i = 0; i < n; i++) {  /* trailers: correct, except every 97th */
            uint32_t c = oracle_crc32(base + off[i], len[i]);
            if (i % 97 == 5) c ^= 1u << (i % 32);
            uint8_t *p = base + off[i] + len[i];
            p[0] = (uint8_t)c, p[1] = (uint8_t)(c >> 8), p[2] = (uint8_t)(c >> 16), p[3] = (uint8_t)(c >> 24);
        }
        const uint32_t s0 = (uint32_t)(r >> 7);
        /* frames: CRC and header_crc */
        if (val_crc32_frames_host(base, base_len, off, len, 0, 0, n, crc, hdr) != VAL_OK) bad("frames_host status", t, it, 0);
        for (uint32_t i = 0; i < n; i++) {
            const uint32_t want = oracle_crc32(base + off[i], len[i]);
            if (crc[i] != want) bad("frames_host crc", t, it, i);
            if (hdr[i] != oracle_crc32(base + off[i], len[i] < 8 ? len[i] : 8)) bad("frames_host hdr", t, it, i);
        }
        /* verify: ok flags, nbad, payload states from a zero register */
        uint32_t nbad = 0, want_bad = 0;
        const val_status_t vs = val_crc32_verify_frames_ex_host(base, base_len, off, len, 0, 0, n, ok, &nbad, pay);
        for (uint32_t i = 0; i < n; i++) {
            const int good = oracle_crc32(base + off[i], len[i]) == le32(base + off[i] + len[i]);
            want_bad += !good;
            if (ok[i] != (uint8_t)good) bad("verify ok", t, it, i);
            const uint8_t *p = base + off[i];
            const uint32_t pre = len[i] >= 8 ? ((p[1] & VAL_DATA_OFFSET_PRESENT) ? 16u : 8u) : UINT32_MAX;
            const uint32_t wp = (len[i] >= 8 && len[i] >= pre) ? oracle_crc32_update_state(0u, p + pre, len[i] - pre) : 0u;
            if (pay[i] != wp) bad("verify pay", t, it, i);
        }
        if (nbad != want_bad || (vs != VAL_OK) != (want_bad != 0)) bad("verify nbad", t, it, nbad);
        /* the multi-device call, CPU route (no device here) */
        memset(crc, 0, n * 4u);
        if (val_crc32_frames_host_multi(base, base_len, off, len, 0, 0, n, crc, NULL, 8) != VAL_OK)
            bad("frames_host_multi status", t, it, 0);
        for (uint32_t i = 0; i < n; i++)
            if (crc[i] != oracle_crc32(base + off[i], len[i])) bad("frames_host_multi crc", t, it, i);
        /* a region window over the whole stream from a seeded state */
        uint32_t st = 0;
        if (val_crc32_region_host_multi(base, base_len, s0, &st, 4) != VAL_OK) bad("region status", t, it, 0);
        if (st != oracle_crc32_update_state(s0, base, base_len)) bad("region state", t, it, base_len);
        /* the scalar hooks on a few frames: the provider (val_config_t.crc32_provider:
           seed 0xFFFFFFFF gives the finished CRC, as stress_provider.c checks)
           and the raw-register update */
        for (uint32_t i = 0; i < n; i += 211) {
            if (val_gpu_crc32_provider(0xFFFFFFFFu, base + off[i], len[i]) != oracle_crc32(base + off[i], len[i]))
                bad("provider", t, it, i);
            if (val_crc32_update_state(s0, base + off[i], len[i]) != oracle_crc32_update_state(s0, base + off[i], len[i]))
                bad("update_state", t, it, i);
        }
        checked += n;
        (void)total;
        free(base), free(off), free(len), free(crc), free(hdr), free(pay), free(ok);
    }
    pthread_mutex_lock(&g_mu);
    g_checked += checked;
    pthread_mutex_unlock(&g_mu);
    return NULL;
}

int main(int argc, char **argv)
{
    const unsigned nth = argc > 1 ? (unsigned)atoi(argv[1]) : 4u;
    g_iters = argc > 2 ? atoi(argv[2]) : 8;
    g_seed = argc > 3 ? strtoull(argv[3], NULL, 0) : 1u;
    val_gpu_set_host_cpu_threads(4);  /* helper threads inside each call as well */
    pthread_t th[64];
    const unsigned k = nth < 64 ? nth : 64;
    for (unsigned t = 0; t < k; t++) pthread_create(&th[t], NULL, worker, (void *)(uintptr_t)t);
    for (unsigned t = 0; t < k; t++) pthread_join(th[t], NULL);
    printf("{\"threads\":%u,\"iters\":%d,\"seed\":%llu,\"frames_checked\":%lu,\"bad\":%lu,\"cpu_batches\":%llu,"
           "\"cpu_fallbacks\":%llu,\"devices\":%d}\n",
           k, g_iters, (unsigned long long)g_seed, g_checked, g_bad, (unsigned long long)val_gpu_cpu_batch_count(),
           (unsigned long long)val_gpu_cpu_fallback_count(), val_gpu_device_count());
    fflush(stdout);
    /* device memory released while the HIP runtime is still loaded (ASAN's
     * device allocator refuses frees that arrive after it has unloaded) */
    val_gpu_shutdown();
    return g_bad ? 1 : 0;
}
