/*
 * val_byte_order.h -- little-endian wire accessors for the frame header and
 * trailer. Byte-wise on every host, so the result never depends on host
 * endianness or alignment (reference include/val_byte_order.h:163-209 keeps
 * a pointer-cast fast path; the bytes on the wire are identical).
 */
#ifndef VAL_BYTE_ORDER_H
#define VAL_BYTE_ORDER_H
#include <stdint.h>

/* forced inlining for the small helpers of VAL's own sources */
#ifndef VAL_FORCE_INLINE
#if defined(__GNUC__) || defined(__clang__)
#define VAL_FORCE_INLINE inline __attribute__((always_inline))
#else
#define VAL_FORCE_INLINE inline
#endif
#endif

static inline void val_put_le16(uint8_t *p, uint16_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); }
static inline void val_put_le32(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}
static inline void val_put_le64(uint8_t *p, uint64_t v)
{
    val_put_le32(p, (uint32_t)v);
    val_put_le32(p + 4, (uint32_t)(v >> 32));
}
static inline uint16_t val_get_le16(const uint8_t *p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static inline uint32_t val_get_le32(const uint8_t *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static inline uint64_t val_get_le64(const uint8_t *p)
{
    return (uint64_t)val_get_le32(p) | ((uint64_t)val_get_le32(p + 4) << 32);
}

#define VAL_PUT_LE16(buf, v) val_put_le16((uint8_t *)(buf), (uint16_t)(v))
#define VAL_PUT_LE32(buf, v) val_put_le32((uint8_t *)(buf), (uint32_t)(v))
#define VAL_PUT_LE64(buf, v) val_put_le64((uint8_t *)(buf), (uint64_t)(v))
#define VAL_GET_LE16(buf) val_get_le16((const uint8_t *)(buf))
#define VAL_GET_LE32(buf) val_get_le32((const uint8_t *)(buf))
#define VAL_GET_LE64(buf) val_get_le64((const uint8_t *)(buf))

#endif /* VAL_BYTE_ORDER_H */
