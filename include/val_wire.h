/*
 * val_wire.h -- VAL v0.7 wire surface (frame layout, control payloads and
 * their codecs, as reference include/val_wire.h) plus the host-side batch
 * framing helpers of the MI355X CRC path.
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

/* Wire sizes of the frame parts and control payloads (reference :14-25). */
#define VAL_WIRE_HEADER_SIZE 8u
#define VAL_WIRE_TRAILER_SIZE 4u
#define VAL_WIRE_HANDSHAKE_SIZE 44u
#define VAL_WIRE_META_SIZE ((VAL_MAX_FILENAME + 1u) + (VAL_MAX_PATH + 1u) + 8u)
#define VAL_WIRE_RESUME_RESP_SIZE 24u
#define VAL_WIRE_VERIFY_REQ_SIZE 16u
#define VAL_WIRE_VERIFY_RESP_SIZE 8u
#define VAL_WIRE_ERROR_PAYLOAD_SIZE 8u
#define VAL_WIRE_VERIFY_REQ_PAYLOAD_SIZE 16u  /* offset u64, crc u32, length u32 */
#define VAL_WIRE_VERIFY_RESP_PAYLOAD_SIZE 8u  /* status i32, receiver crc u32 */
#define VAL_FRAME_HEADER_SIZE VAL_WIRE_HEADER_SIZE
#define VAL_FRAME_TRAILER_SIZE VAL_WIRE_TRAILER_SIZE
#define VAL_WIRE_MAX_CONTENT 0xFFFFu /* content_len is a 16-bit field */

/* RESUME / VERIFY option bits (reserved by v0.7) */
#define VAL_RESUMERESP_VERIFY_REQUIRED (1u << 0)
#define VAL_RESUMERESP_HAS_VERIFY_WINDOW (1u << 1)
#define VAL_VERIFY_REQUEST (1u << 0)

/* DATA flags (byte 1): OFFSET_PRESENT = content starts with the LE64 file offset */
#define VAL_DATA_OFFSET_PRESENT (1u << 0)
#define VAL_DATA_FINAL_CHUNK (1u << 1)
/* DATA_ACK flags */
#define VAL_ACK_FEEDBACK_PRESENT (1u << 0)
#define VAL_ACK_DONE_FILE (1u << 1)
#define VAL_ACK_EOT (1u << 2)

/* HELLO payload, host form (wire: 44 bytes, little-endian, by the codec
 * below; reference :53-75). The window fields carry the flow-control
 * capabilities; the negotiated window is the natural batch size of the
 * GPU TX/RX calls. */
typedef struct {
    uint32_t magic;
    uint8_t version_major;
    uint8_t version_minor;
    uint16_t reserved;
    uint32_t packet_size;
    uint32_t features;
    uint32_t required;
    uint32_t requested;
    uint16_t tx_max_window_packets;
    uint16_t rx_max_window_packets;
    uint8_t ack_stride_packets; /* 0 = one ACK per window */
    uint8_t reserved_capabilities[3];
    uint16_t supported_features16;
    uint16_t required_features16;
    uint16_t requested_features16;
    uint32_t reserved2;
} val_handshake_t;

/* ERROR payload (wire: code i32, detail u32). */
typedef struct {
    int32_t code;
    uint32_t detail;
} val_error_payload_t;

/* Control codecs, same signatures and bytes as the reference
 * (include/val_wire.h:86-105, src/val_wire.c); NULL arguments are no-ops. */
void val_serialize_frame_header(uint8_t type, uint8_t flags, uint16_t content_len, uint32_t type_data, uint8_t *wiredata);
void val_deserialize_frame_header(const uint8_t *wiredata, uint8_t *type, uint8_t *flags, uint16_t *content_len,
                                  uint32_t *type_data);
void val_serialize_handshake(const val_handshake_t *hs, uint8_t *wire_data);
void val_deserialize_handshake(const uint8_t *wire_data, val_handshake_t *hs);
void val_serialize_meta(const val_meta_payload_t *meta, uint8_t *wire_data);
void val_deserialize_meta(const uint8_t *wire_data, val_meta_payload_t *meta);
void val_serialize_resume_resp(const val_resume_resp_t *resp, uint8_t *wire_data);
void val_deserialize_resume_resp(const uint8_t *wire_data, val_resume_resp_t *resp);
void val_serialize_verify_request(uint64_t offset, uint32_t crc, uint32_t length, uint8_t *wire_data);
void val_deserialize_verify_request(const uint8_t *wire_data, uint64_t *offset, uint32_t *crc, uint32_t *length);
void val_serialize_verify_response(val_status_t result, uint32_t receiver_crc, uint8_t *wire_data);
void val_deserialize_verify_response(const uint8_t *wire_data, val_status_t *result, uint32_t *receiver_crc);
void val_serialize_error_payload(const val_error_payload_t *payload, uint8_t *wire_data);
void val_deserialize_error_payload(const uint8_t *wire_data, val_error_payload_t *payload);

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

/*
 * File offset of each scanned frame as the receiver reads it (reference
 * src/val_core.c:981-993): the LE64 after the header for a DATA frame with
 * VAL_DATA_OFFSET_PRESENT, VAL_FRAME_OFFSET_IMPLIED for a DATA frame without
 * it (the receiver's current position), VAL_FRAME_OFFSET_NOT_DATA for other
 * frames (and a DATA frame too short to hold its offset). Pairs with
 * val_crc32_fold_payload_states_at.
 */
#define VAL_FRAME_OFFSET_IMPLIED UINT64_MAX
#define VAL_FRAME_OFFSET_NOT_DATA (UINT64_MAX - 1u)
void val_frame_data_offsets(const uint8_t *stream, const uint64_t *frame_off, const uint32_t *crc_len, uint32_t n,
                            uint64_t *file_off);

#ifdef __cplusplus
}
#endif
#endif /* VAL_WIRE_H */
