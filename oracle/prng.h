/*
 * Deterministic synthetic payload bytes shared by the golden generator, the
 * tests (numpy restatement in tests/_prng.py) and bench.py.
 * TEST INFRASTRUCTURE. byte i of stream `seed` = LE byte (i % 8) of
 * splitmix64(seed + (i/8 + 1) * 0x9E3779B97F4A7C15).
 */
#ifndef VAL_ORACLE_PRNG_H
#define VAL_ORACLE_PRNG_H
#include <stddef.h>
#include <stdint.h>
static inline uint64_t oracle_splitmix64(uint64_t seed, uint64_t k)
{
    uint64_t z = seed + (k + 1u) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline void oracle_prng_fill(uint64_t seed, uint8_t *out, size_t n)
{
    for (size_t i = 0; i < n; i++)
        out[i] = (uint8_t)(oracle_splitmix64(seed, i / 8u) >> (8u * (i % 8u)));
}
#endif
