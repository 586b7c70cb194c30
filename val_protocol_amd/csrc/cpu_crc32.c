/*
 * cpu_crc32.c -- this library's own host CRC-32 (C99 + x86 intrinsics).
 *
 * Used by the three scalar hooks (val_gpu_crc32_provider, val_crc32,
 * val_crc32_update_state) for inputs below the provider threshold, where a
 * GPU round trip (~18 us of launch + completion) cannot win, and as their
 * failure fallback. Never used by the batch or device calls.
 *
 * Same function as the reference's byte loop (src/val_core.c:150-160):
 * the raw reflected register advanced over the bytes, no init/xorout here.
 * Two engines, both built from gf2_crc32.h at first use (not the oracle):
 *   - slice-by-16: T_k[b] = b * x^(8(k+1)) mod P, 16 bytes per step
 *     (T_0 is the reference's table, src/val_core.c:133-148);
 *   - carry-less multiply folding (x86 PCLMULQDQ, runtime-detected) for
 *     inputs of >= 64 bytes: four 16-byte accumulators are advanced over 64
 *     bytes per step by multiplying each half by x^e mod P, then folded into
 *     one 16-byte value congruent to everything hashed so far; that value and
 *     the tail go through slice-by-16. No Barrett step is needed;
 *   - the same folding on 512-bit registers (VPCLMULQDQ + AVX-512F, e.g.
 *     Zen 4/5 hosts of MI355X), 256 bytes per step, for inputs >= 256 bytes.
 *
 * Representation (see gf2_crc32.h): register bit i = coefficient of x^(31-i).
 * A 16-byte block loaded little-endian has bit k (bit k%8 of byte k/8, the
 * k-th bit on the wire) = coefficient of x^(127-k). The carry-less product
 * of 64-bit halves a, b read that way is x * A(x) * B(x), so the constant
 * for "multiply by x^e" is x^(e-1) mod P placed in the top 32 bits.
 */
#include "cpu_crc32.h"

#include <pthread.h>
#include <stdint.h>
#include <string.h>

#include "gf2_crc32.h"

#if defined(__x86_64__)
#include <immintrin.h>
#define VCRC_HAVE_CLMUL_BUILD 1
#endif

static uint32_t g_t16[16][256];
static int g_use_clmul;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

/* x^e mod P as a register */
static uint32_t xpow(uint64_t e)
{
    return gf2_mul(gf2_x8n(e >> 3), GF2_ONE >> (e & 7u));
}

#ifdef VCRC_HAVE_CLMUL_BUILD
/* {multiplier of the first 8 bytes, multiplier of the last 8} of a block
 * advanced over d bytes: x^(64 + 8d) and x^(8d), as carry-less constants */
static uint64_t g_fold[4][2]; /* d = 16, 32, 48, 64 */
static uint64_t g_fold_wide[4][2]; /* d = 64, 128, 192, 256 (512-bit lanes) */
static int g_use_vpclmul;

static uint64_t clmul_const(uint64_t e) { return (uint64_t)xpow(e - 1u) << 32; }
#endif

static void init_tables(void)
{
    for (int k = 0; k < 16; k++) {
        const uint32_t xk = gf2_x8n((uint64_t)(k + 1));
        for (int b = 0; b < 256; b++)
            g_t16[k][b] = gf2_mul(xk, (uint32_t)b);
    }
#ifdef VCRC_HAVE_CLMUL_BUILD
    for (int i = 0; i < 4; i++) {
        const uint64_t d = 16u * (uint64_t)(i + 1);
        g_fold[i][0] = clmul_const(64u + 8u * d);
        g_fold[i][1] = clmul_const(8u * d);
        g_fold_wide[i][0] = clmul_const(64u + 32u * d);
        g_fold_wide[i][1] = clmul_const(32u * d);
    }
    __builtin_cpu_init();
    g_use_clmul = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
    g_use_vpclmul = g_use_clmul && __builtin_cpu_supports("vpclmulqdq") && __builtin_cpu_supports("avx512f");
#endif
}

static uint32_t slice16(uint32_t c, const uint8_t *p, size_t len)
{
    while (len >= 16) {
        uint32_t w[4];
        memcpy(w, p, 16);
        w[0] ^= c;
        c = g_t16[15][w[0] & 0xFF] ^ g_t16[14][(w[0] >> 8) & 0xFF] ^ g_t16[13][(w[0] >> 16) & 0xFF] ^
            g_t16[12][w[0] >> 24] ^ g_t16[11][w[1] & 0xFF] ^ g_t16[10][(w[1] >> 8) & 0xFF] ^
            g_t16[9][(w[1] >> 16) & 0xFF] ^ g_t16[8][w[1] >> 24] ^ g_t16[7][w[2] & 0xFF] ^
            g_t16[6][(w[2] >> 8) & 0xFF] ^ g_t16[5][(w[2] >> 16) & 0xFF] ^ g_t16[4][w[2] >> 24] ^
            g_t16[3][w[3] & 0xFF] ^ g_t16[2][(w[3] >> 8) & 0xFF] ^ g_t16[1][(w[3] >> 16) & 0xFF] ^
            g_t16[0][w[3] >> 24];
        p += 16;
        len -= 16;
    }
    while (len--)
        c = g_t16[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
    return c;
}

#ifdef VCRC_HAVE_CLMUL_BUILD
__attribute__((target("pclmul,sse4.1"))) static inline __m128i fold(__m128i x, __m128i k)
{
    return _mm_xor_si128(_mm_clmulepi64_si128(x, k, 0x00), _mm_clmulepi64_si128(x, k, 0x11));
}

/* 512-bit form: the same fold on four 16-byte lanes at once */
__attribute__((target("vpclmulqdq,avx512f"))) static inline __m512i fold512(__m512i x, __m512i k)
{
    return _mm512_xor_si512(_mm512_clmulepi64_epi128(x, k, 0x00), _mm512_clmulepi64_epi128(x, k, 0x11));
}

__attribute__((target("vpclmulqdq,avx512f"))) static inline __m512i wide_const(int i)
{
    return _mm512_broadcast_i32x4(_mm_set_epi64x((long long)g_fold_wide[i][1], (long long)g_fold_wide[i][0]));
}

/* len >= 256: four 64-byte accumulators over 256 bytes per step, folded to one
 * 64-byte accumulator, then to 16 bytes (lane j advanced over 48 - 16 j). */
__attribute__((target("vpclmulqdq,avx512f,pclmul,sse4.1"))) static uint32_t vpclmul_update(uint32_t c, const uint8_t *p,
                                                                                         size_t len)
{
    const __m512i k64 = wide_const(0), k128 = wide_const(1), k192 = wide_const(2), k256 = wide_const(3);
    __m512i z0 = _mm512_loadu_si512((const void *)p);
    __m512i z1 = _mm512_loadu_si512((const void *)(p + 64));
    __m512i z2 = _mm512_loadu_si512((const void *)(p + 128));
    __m512i z3 = _mm512_loadu_si512((const void *)(p + 192));
    z0 = _mm512_xor_si512(z0, _mm512_zextsi128_si512(_mm_cvtsi32_si128((int)c)));
    p += 256;
    len -= 256;
    while (len >= 256) {
        z0 = _mm512_xor_si512(fold512(z0, k256), _mm512_loadu_si512((const void *)p));
        z1 = _mm512_xor_si512(fold512(z1, k256), _mm512_loadu_si512((const void *)(p + 64)));
        z2 = _mm512_xor_si512(fold512(z2, k256), _mm512_loadu_si512((const void *)(p + 128)));
        z3 = _mm512_xor_si512(fold512(z3, k256), _mm512_loadu_si512((const void *)(p + 192)));
        p += 256;
        len -= 256;
    }
    __m512i z = _mm512_xor_si512(_mm512_xor_si512(fold512(z0, k192), fold512(z1, k128)),
                                 _mm512_xor_si512(fold512(z2, k64), z3));
    while (len >= 64) {
        z = _mm512_xor_si512(fold512(z, k64), _mm512_loadu_si512((const void *)p));
        p += 64;
        len -= 64;
    }
    const __m128i k16 = _mm_set_epi64x((long long)g_fold[0][1], (long long)g_fold[0][0]);
    const __m128i k32 = _mm_set_epi64x((long long)g_fold[1][1], (long long)g_fold[1][0]);
    const __m128i k48 = _mm_set_epi64x((long long)g_fold[2][1], (long long)g_fold[2][0]);
    __m128i v = _mm_xor_si128(_mm_xor_si128(fold(_mm512_extracti32x4_epi32(z, 0), k48),
                                            fold(_mm512_extracti32x4_epi32(z, 1), k32)),
                              _mm_xor_si128(fold(_mm512_extracti32x4_epi32(z, 2), k16), _mm512_extracti32x4_epi32(z, 3)));
    while (len >= 16) {
        v = _mm_xor_si128(fold(v, k16), _mm_loadu_si128((const __m128i *)(const void *)p));
        p += 16;
        len -= 16;
    }
    uint8_t blk[16];
    _mm_storeu_si128((__m128i *)(void *)blk, v);
    return slice16(slice16(0u, blk, 16), p, len);
}

/* len >= 64 */
__attribute__((target("pclmul,sse4.1"))) static uint32_t clmul_update(uint32_t c, const uint8_t *p, size_t len)
{
    const __m128i k16 = _mm_set_epi64x((long long)g_fold[0][1], (long long)g_fold[0][0]);
    const __m128i k32 = _mm_set_epi64x((long long)g_fold[1][1], (long long)g_fold[1][0]);
    const __m128i k48 = _mm_set_epi64x((long long)g_fold[2][1], (long long)g_fold[2][0]);
    const __m128i k64 = _mm_set_epi64x((long long)g_fold[3][1], (long long)g_fold[3][0]);
    __m128i a0 = _mm_loadu_si128((const __m128i *)(const void *)p);
    __m128i a1 = _mm_loadu_si128((const __m128i *)(const void *)(p + 16));
    __m128i a2 = _mm_loadu_si128((const __m128i *)(const void *)(p + 32));
    __m128i a3 = _mm_loadu_si128((const __m128i *)(const void *)(p + 48));
    /* the initial register is the first 4 bytes XORed with it, from zero */
    a0 = _mm_xor_si128(a0, _mm_cvtsi32_si128((int)c));
    p += 64;
    len -= 64;
    while (len >= 64) {
        a0 = _mm_xor_si128(fold(a0, k64), _mm_loadu_si128((const __m128i *)(const void *)p));
        a1 = _mm_xor_si128(fold(a1, k64), _mm_loadu_si128((const __m128i *)(const void *)(p + 16)));
        a2 = _mm_xor_si128(fold(a2, k64), _mm_loadu_si128((const __m128i *)(const void *)(p + 32)));
        a3 = _mm_xor_si128(fold(a3, k64), _mm_loadu_si128((const __m128i *)(const void *)(p + 48)));
        p += 64;
        len -= 64;
    }
    __m128i v = _mm_xor_si128(_mm_xor_si128(fold(a0, k48), fold(a1, k32)), _mm_xor_si128(fold(a2, k16), a3));
    while (len >= 16) {
        v = _mm_xor_si128(fold(v, k16), _mm_loadu_si128((const __m128i *)(const void *)p));
        p += 16;
        len -= 16;
    }
    uint8_t blk[16];
    _mm_storeu_si128((__m128i *)(void *)blk, v);
    return slice16(slice16(0u, blk, 16), p, len);
}
#endif

uint32_t vcrc_cpu_update_with(int engine, uint32_t state, const void *data, size_t len)
{
    pthread_once(&g_once, init_tables);
    const uint8_t *p = (const uint8_t *)data;
    if (engine == VCRC_CPU_BEST)
        engine = g_use_vpclmul ? VCRC_CPU_VPCLMUL : g_use_clmul ? VCRC_CPU_CLMUL : VCRC_CPU_SLICE16;
#ifdef VCRC_HAVE_CLMUL_BUILD
    if (engine == VCRC_CPU_VPCLMUL && g_use_vpclmul && len >= 256)
        return vpclmul_update(state, p, len);
    if (engine >= VCRC_CPU_CLMUL && g_use_clmul && len >= 64)
        return clmul_update(state, p, len);
#endif
    return slice16(state, p, len);
}

uint32_t vcrc_cpu_update(uint32_t state, const void *data, size_t len)
{
    return vcrc_cpu_update_with(VCRC_CPU_BEST, state, data, len);
}

int vcrc_cpu_engine(void)
{
    pthread_once(&g_once, init_tables);
    return g_use_vpclmul ? VCRC_CPU_VPCLMUL : g_use_clmul ? VCRC_CPU_CLMUL : VCRC_CPU_SLICE16;
}
