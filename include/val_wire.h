/*
 * val_wire.h -- VAL v0.7 frame layout and the host-side framing helpers of
 * the MI355X CRC path.
 *
 * Frame (reference include/val_wire.h:14,21,32-38):
 *   [0] type  [1] flags  [2..3] content_len LE16  [4..7] type_data LE32
 *   [8 .. 8+content_len)  content   (DATA + OFFSET_PRESENT: LE64 offset, payload)
 *   [8+content_len .. +4) trailer = LE32 CRC-32 over bytes [0, 8+content_len)
 *
 * "CRC input" of a frame = its first 8 + content_len bytes.
 * header_crc (this build's definition): CRC-32 of the
 * 8 header bytes, i.e. the finished CRC of the first 8 bytes of the CRC input.
 */
#ifndef VAL_WIRE_H
#define VAL_WIRE_H

#include <stddef.h>
#include <stdint.h>

#include "val_protocol.h"

#ifdef __cplusplus
extern "C" {
#endif

#define VAL_WIRE_HEADER_SIZE 8u
#define VAL_WIRE_TRAILER_SIZE 4u
#define VAL_FRAME_HEADER_SIZE VAL_WIRE_HEADER_SIZE
#define VAL_FRAME_TRAILER_SIZE VAL_WIRE_TRAILER_SIZE
#define VAL_WIRE_MAX_CONTENT 0xFFFFu /* content_len is a 16-bit field */

#define VAL_DATA_OFFSET_PRESENT (1u << 0)
#define VAL_DATA_FINAL_CHUNK (1u << 1)
#define VAL_ACK_FEEDBACK_PRESENT (1u << 0)
#define VAL_ACK_DONE_FILE (1u << 1)
#define VAL_ACK_EOT (1u << 2)

/* Same signatures as the reference codec (include/val_wire.h:86-87). */
void val_serialize_frame_header(uint8_t type, uint8_t flags, uint16_t content_len, uint32_t type_data, uint8_t *wiredata);
void val_deserialize_frame_header(const uint8_t *wiredata, uint8_t *type, uint8_t *flags, uint16_t *content_len,
                                  uint32_t *type_data);

/*
 * TX batch framing (the window-fill loop of src/val_sender.c:822-841 turned
 * into one staging pass). Lays `n` DATA frames back to back
 * in `out`: frame i carries payload bytes [pay_off[i], pay_off[i]+pay_len[i])
 * of `payload`, file offset file_off[i], and an LE64 offset prefix when
 * include_offset[i] != 0 (NULL = all explicit, as val_internal_send_packet).
 * Trailers are left zero for the GPU kernel to fill. Writes each frame's
 * start into frame_off[i] and its CRC-input length into crc_len[i].
 * Unlike the reference (src/val_core.c:747, which silently truncates), a
 * content_len above 65535 is rejected with VAL_ERR_INVALID_ARG.
 * *out_used receives the bytes written.
 */
val_status_t val_frame_data_batch(const uint8_t *payload, const uint64_t *pay_off, const uint32_t *pay_len,
                                  const uint64_t *file_off, const uint8_t *include_offset, uint32_t n, uint8_t *out,
                                  size_t out_cap, uint64_t *frame_off, uint32_t *crc_len, size_t *out_used);

/* Write LE32 trailers crc[i] after each frame's CRC input. */
void val_frame_put_trailers(uint8_t *stream, const uint64_t *frame_off, const uint32_t *crc_len, const uint32_t *crc,
                            uint32_t n);

/*
 * RX batch scan: walk a byte stream of concatenated frames (what the
 * receiver's transport delivered) and emit descriptors for the batch verify
 * kernel. Stops at the first incomplete frame or after `max_frames`, or when
 * a header announces content beyond `mtu` - 12 (reference check at
 * src/val_core.c:915-921 -> VAL_ERR_PROTOCOL). *n_frames / *consumed report
 * what was parsed.
 */
val_status_t val_frame_scan(const uint8_t *stream, size_t len, size_t mtu, uint32_t max_frames, uint64_t *frame_off,
                            uint32_t *crc_len, uint32_t *n_frames, size_t *consumed);

/*
 * Payload length of each scanned frame: CRC input minus the 8-byte header
 * and, when flags has VAL_DATA_OFFSET_PRESENT, the 8-byte file offset (the
 * bytes the receiver writes and feeds to its rolling CRC, reference
 * src/val_receiver.c:880-891); 0 for a frame shorter than that prefix.
 * Pairs with the payload states of val_crc32_verify_frames_ex_*.
 */
void val_frame_payload_lens(const uint8_t *stream, const uint64_t *frame_off, const uint32_t *crc_len, uint32_t n,
                            uint32_t *pay_len);

#ifdef __cplusplus
}
#endif
#endif /* VAL_WIRE_H */
