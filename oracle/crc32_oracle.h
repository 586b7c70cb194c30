/*
 * crc32_oracle.h -- CPU restatement of VAL v0.7's CRC-32 integrity path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * or the timed CPU baseline.  The product (val_protocol_amd/libval_crc_hip.so)
 * never links or calls it.
 *
 * Parity is pinned two ways (see DESIGN.md "Oracle"):
 *   1. against golden vectors in tests/golden/ produced by the reference
 *      library itself (oracle/_ref/libval_ref.so, built from
 *      /root/reference/src by oracle/Makefile), and
 *   2. against the published CRC-32/ISO-HDLC check value 0xCBF43926
 *      (/root/reference/docs/message-formats.md:461-466).
 */
#ifndef VAL_CRC32_ORACLE_H
#define VAL_CRC32_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Byte-at-a-time table CRC, reflected poly 0xEDB88320
 * (reference: src/val_core.c:129-160). Finalized (xorout 0xFFFFFFFF). */
uint32_t oracle_crc32(const void *data, size_t len);
/* Raw-register incremental form (src/val_core.c:162-183). */
uint32_t oracle_crc32_init_state(void);
uint32_t oracle_crc32_update_state(uint32_t state, const void *data, size_t len);
uint32_t oracle_crc32_finalize_state(uint32_t state);
/* crc32_func_t semantics (include/val_protocol.h:163-166, resolved per
 * SURVEY.md 8(b)): finalize(update(seed, buf, len)). */
uint32_t oracle_crc32_provider(uint32_t seed, const void *buf, size_t len);

/* GF(2) algebra: register * x^(8n) mod P (advance by n zero bytes), and the
 * standard combine crc(A||B) from crc(A), crc(B), |B|. Not in the reference;
 * restated from the published CRC algebra (zlib crc32_combine identity). */
uint32_t oracle_crc32_shift(uint32_t state, uint64_t nbytes);
uint32_t oracle_crc32_combine(uint32_t crc_a, uint32_t crc_b, uint64_t len_b);

/* TX framing of one DATA packet exactly as val__internal_send_packet_core
 * (src/val_core.c:718-866): header [5, flags, LE16 content_len, LE32 0],
 * optional LE64 offset prefix, payload, LE32 trailer CRC over header+content.
 * content_len is truncated to 16 bits as at src/val_core.c:747.
 * Returns the wire length, or 0 if out_cap is too small. */
size_t oracle_build_data_frame(const uint8_t *payload, uint32_t payload_len, uint64_t offset,
                               int include_offset, uint8_t *out, size_t out_cap);

/* Per-frame batch form (the loop a sender/receiver runs once per frame):
 * crc[i] = CRC32(base[off[i] .. off[i]+len[i])), hdr[i] = CRC32(first 8 bytes)
 * (hdr may be NULL). nthreads>1 splits frames round-robin over pthreads. */
void oracle_crc32_frames(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t n,
                         uint32_t *crc, uint32_t *hdr, int nthreads);
/* Uniform strided batch: frame i at base + i*stride, CRC over flen bytes. */
void oracle_crc32_frames_strided(const uint8_t *base, uint64_t stride, uint32_t flen, uint64_t n,
                                 uint32_t *crc, uint32_t *hdr, int nthreads);
/* RX verify (src/val_core.c:963-974): ok[i] = (crc == LE32 trailer after the
 * CRC input). Returns the number of mismatches (the crc_errors increments). */
uint64_t oracle_verify_frames(const uint8_t *base, const uint64_t *off, const uint32_t *len, uint64_t n,
                              uint8_t *ok, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
