/*
 * gf2_crc32.h -- GF(2)[x] / P arithmetic for CRC-32/ISO-HDLC in the
 * reflected representation (bit 31 of a register = coefficient of x^0,
 * P = 0xEDB88320 reflected). Shared by host and device code.
 *
 * Facts the kernels rely on (all linear over GF(2)):
 *   advance(r, n zero bytes) = gf2_mul(gf2_x8n(n), r)
 *   state(A||B from r)      = advance(state(A from r), |B|) ^ state(B from 0)
 *   byte table T_k[b]        = gf2_mul(gf2_x8n(k+1), b)   (T_0 = classic table,
 *                              reference src/val_core.c:133-148)
 */
#ifndef VAL_GF2_CRC32_H
#define VAL_GF2_CRC32_H
#include <stdint.h>

#if defined(__HIPCC__)
#define GF2_FN __host__ __device__ __forceinline__
#else
#define GF2_FN static inline
#endif

#define GF2_POLY 0xEDB88320u
#define GF2_ONE 0x80000000u /* x^0 */

/* a * b mod P */
GF2_FN uint32_t gf2_mul(uint32_t a, uint32_t b)
{
    uint32_t prod = 0;
    for (int i = 31; i >= 0; i--) {
        prod ^= (0u - ((a >> i) & 1u)) & b;
        b = (b >> 1) ^ ((0u - (b & 1u)) & GF2_POLY);
    }
    return prod;
}

/* x^(8n) mod P */
GF2_FN uint32_t gf2_x8n(uint64_t n)
{
    uint32_t result = GF2_ONE, sq = 0x00800000u; /* x^8 */
    while (n) {
        if (n & 1u) result = gf2_mul(result, sq);
        sq = gf2_mul(sq, sq);
        n >>= 1;
    }
    return result;
}

#endif /* VAL_GF2_CRC32_H */
