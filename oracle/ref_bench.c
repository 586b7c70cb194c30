/*
 * ref_bench.c -- CPU baseline driver (TEST/BENCH INFRASTRUCTURE).
 * Times the REFERENCE val_crc32 (oracle/_ref/libval_ref.so, built from
 * /root/reference/src/val_core.c:150-160) over a batch of frames with
 * pthreads, frames round-robin per thread, as SURVEY.md 8(d) prescribes.
 */
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>

uint32_t val_crc32(const void *data, size_t length); /* from libval_ref.so */

typedef struct {
    const uint8_t *base;
    uint64_t stride, n;
    uint32_t flen;
    const uint64_t *off; /* descriptor mode (NULL: strided) */
    const uint32_t *len;
    uint32_t *out;
    int tid, nth;
} job_t;

static void *run(void *a)
{
    job_t *j = (job_t *)a;
    for (uint64_t i = (uint64_t)j->tid; i < j->n; i += (uint64_t)j->nth)
        j->out[i] = j->off ? val_crc32(j->base + j->off[i], j->len[i]) : val_crc32(j->base + i * j->stride, j->flen);
    return NULL;
}

static void run_all(job_t proto, int nthreads)
{
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    job_t jobs[256];
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = proto;
        jobs[t].tid = t;
        jobs[t].nth = nthreads;
        if (nthreads > 1) pthread_create(&th[t], NULL, run, &jobs[t]);
        else run(&jobs[t]);
    }
    for (int t = 0; nthreads > 1 && t < nthreads; t++) pthread_join(th[t], NULL);
}

void ref_bench_frames(const uint8_t *base, uint64_t stride, uint32_t flen, uint64_t n, uint32_t *out, int nthreads)
{
    job_t j = {base, stride, n, flen, NULL, NULL, out, 0, 1};
    run_all(j, nthreads);
}

/* Ragged batches (cfg5): frame i = base[off[i], off[i] + len[i]). */
void ref_bench_frames_desc(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t n, uint32_t *out,
                           int nthreads)
{
    job_t j = {base, 0, n, 0, off, len, out, 0, 1};
    run_all(j, nthreads);
}
