/* Stress the scalar provider hook (TEST INFRASTRUCTURE): N calls of
 * val_gpu_crc32_provider on random lengths / alignments / data from one
 * reused malloc buffer, against the CPU oracle. Prints mismatches.
 * usage: stress_provider N seed [lo hi] */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "crc32_oracle.h"
#include "prng.h"
#include "val_crc32_gpu.h"

int main(int argc, char **argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 1000;
    uint64_t seed = argc > 2 ? strtoull(argv[2], 0, 0) : 1;
    const uint32_t lo = argc > 3 ? (uint32_t)atoi(argv[3]) : 1, hi = argc > 4 ? (uint32_t)atoi(argv[4]) : 70000;
    uint8_t *buf = malloc(hi + 64);
    int bad = 0;
    for (int i = 0; i < n; i++) {
        uint64_t r = seed * 0x9E3779B97F4A7C15ull + (uint64_t)i * 0xD1B54A32D192ED03ull;
        r ^= r >> 31;
        const uint32_t len = lo + (uint32_t)(r % (hi - lo + 1));
        const uint32_t al = (uint32_t)((r >> 40) & 15);
        oracle_prng_fill(r, buf + al, len);
        const uint32_t want = oracle_crc32(buf + al, len);
        const uint32_t got = val_gpu_crc32_provider(0xFFFFFFFFu, buf + al, len);
        if (got != want) {
            if (bad < 20) printf("BAD i=%d len=%u align=%u got=%08x want=%08x\n", i, len, al, got, want);
            bad++;
        }
    }
    printf("stress_provider n=%d seed=%llu bad=%d\n", n, (unsigned long long)seed, bad);
    return bad ? 1 : 0;
}
