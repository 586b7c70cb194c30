/* Per-call cost of the scalar CRC hook at VAL frame sizes (measurement tool,
 * test infrastructure): the product's val_gpu_crc32_provider (its CPU engine
 * below the provider threshold) against the reference's own val_crc32
 * (src/val_core.c:150-160, compiled into oracle/_ref/libval_ref.so), called
 * from C in a loop over a buffer that stays in cache, so the figures carry no
 * binding overhead. Prints one JSON line per size; with a thread count, the
 * same calls from that many threads at once (concurrent sessions), as
 * aggregate calls per second.
 * usage: provider_bench <libval_crc_hip.so> <libval_ref.so> [threads] */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "prng.h"

typedef uint32_t (*prov_t)(uint32_t, const void *, size_t);
typedef uint32_t (*crc_t)(const void *, size_t);

static double now_ns(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e9 + t.tv_nsec;
}

static prov_t g_prov;
static crc_t g_ref;
static size_t g_n;
static long g_reps;
static int g_which;

static void *worker(void *arg)
{
    uint8_t buf[1 << 12];
    oracle_prng_fill((uint64_t)(uintptr_t)arg, buf, sizeof buf);
    uint32_t s = 0;
    for (long i = 0; i < g_reps; i++)
        s ^= g_which ? g_ref(buf + (i & 63), g_n) : g_prov(0xFFFFFFFFu, buf + (i & 63), g_n);
    return (void *)(uintptr_t)s;
}

/* Aggregate calls/s of T threads calling one hook on g_n bytes. */
static double threaded(int T, int which, size_t n, long reps)
{
    pthread_t th[64];
    g_which = which;
    g_n = n;
    g_reps = reps;
    const double t0 = now_ns();
    for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, worker, (void *)(uintptr_t)(t + 1));
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    return (double)T * reps / ((now_ns() - t0) * 1e-9);
}

int main(int argc, char **argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: %s <libval_crc_hip.so> <libval_ref.so>\n", argv[0]);
        return 2;
    }
    void *lp = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL), *lr = dlopen(argv[2], RTLD_NOW | RTLD_LOCAL);
    if (!lp || !lr) {
        fprintf(stderr, "dlopen: %s\n", dlerror());
        return 2;
    }
    prov_t prov = (prov_t)dlsym(lp, "val_gpu_crc32_provider");
    crc_t ref = (crc_t)dlsym(lr, "val_crc32");
    if (!prov || !ref) return 2;
    static const size_t sizes[] = {16, 64, 256, 1040, 4104, 16400, 65532, 65543};
    uint8_t *buf = malloc(1 << 17);
    oracle_prng_fill(0x5EED, buf, 1 << 17);
    for (size_t k = 0; k < sizeof sizes / sizeof sizes[0]; k++) {
        const size_t n = sizes[k];
        const long reps = (long)(2e8 / (n + 64));
        uint32_t sink = 0;
        if (prov(0xFFFFFFFFu, buf, n) != ref(buf, n)) {
            fprintf(stderr, "mismatch at %zu\n", n);
            return 1;
        }
        double best_p = 1e30, best_r = 1e30;
        for (int r = 0; r < 5; r++) {
            double t0 = now_ns();
            for (long i = 0; i < reps; i++) sink ^= prov(0xFFFFFFFFu, buf + (i & 63), n);
            double t1 = now_ns();
            for (long i = 0; i < reps / 8 + 1; i++) sink ^= ref(buf + (i & 63), n);
            double t2 = now_ns();
            if ((t1 - t0) / reps < best_p) best_p = (t1 - t0) / reps;
            if ((t2 - t1) / (reps / 8 + 1) < best_r) best_r = (t2 - t1) / (reps / 8 + 1);
        }
        printf("{\"bytes\": %zu, \"product_ns\": %.1f, \"reference_ns\": %.1f, \"speedup\": %.1f, \"product_GiB_s\": %.2f, "
               "\"reference_GiB_s\": %.3f, \"sink\": %u}\n",
               n, best_p, best_r, best_r / best_p, n / best_p / 1.073741824, n / best_r / 1.073741824, sink & 1u);
    }
    free(buf);
    const int T = argc > 3 ? atoi(argv[3]) : 0;
    if (T > 0 && T <= 64) {
        g_prov = prov;
        g_ref = ref;
        static const size_t tsz[] = {16, 1040};
        for (int k = 0; k < 2; k++) {
            double p1 = 0, pt = 0, rt = 0;
            for (int r = 0; r < 3; r++) {
                const double a = threaded(1, 0, tsz[k], 4000000), b = threaded(T, 0, tsz[k], 4000000),
                             c = threaded(T, 1, tsz[k], tsz[k] > 64 ? 100000 : 2000000);
                p1 = a > p1 ? a : p1;
                pt = b > pt ? b : pt;
                rt = c > rt ? c : rt;
            }
            printf("{\"bytes\": %zu, \"threads\": %d, \"product_calls_per_s_1thread\": %.3g, "
                   "\"product_calls_per_s\": %.3g, \"reference_calls_per_s\": %.3g, \"product_scaling\": %.2f}\n",
                   tsz[k], T, p1, pt, rt, pt / p1);
        }
    }
    return 0;
}
