/*
 * val_wire.c -- host-side frame codec and batch framing for the MI355X CRC
 * path (C99). The GPU kernels hash what these helpers lay out.
 *
 * Header and control codecs: same byte layouts as the reference
 * (src/val_wire.c:27-192).
 * Batch framing: the per-frame body of val__internal_send_packet_core
 * (src/val_core.c:733-832) applied to a whole window of DATA frames at once,
 * so one kernel launch can fill every trailer.
 * Stream scan: the header/length checks of val_internal_recv_packet
 * (src/val_core.c:893-921) applied to a buffered byte stream (8(f) f2).
 */
#include <string.h>

#include "val_byte_order.h"
#include "val_wire.h"

void val_serialize_frame_header(uint8_t type, uint8_t flags, uint16_t content_len, uint32_t type_data, uint8_t *wiredata)
{
    if (!wiredata)
        return;
    wiredata[0] = type;
    wiredata[1] = flags;
    val_put_le16(wiredata + 2, content_len);
    val_put_le32(wiredata + 4, type_data);
}

void val_deserialize_frame_header(const uint8_t *wiredata, uint8_t *type, uint8_t *flags, uint16_t *content_len,
                                  uint32_t *type_data)
{
    if (!wiredata)
        return;
    if (type)
        *type = wiredata[0];
    if (flags)
        *flags = wiredata[1];
    if (content_len)
        *content_len = val_get_le16(wiredata + 2);
    if (type_data)
        *type_data = val_get_le32(wiredata + 4);
}

/* ---- control payload codecs: field by field, little-endian (the byte
 * layouts of reference src/val_wire.c:47-192; pinned by
 * tests/test_header_surface.py against the reference's own codec). */
void val_serialize_handshake(const val_handshake_t *hs, uint8_t *wire_data)
{
    if (!hs || !wire_data)
        return;
    uint8_t *w = wire_data;
    val_put_le32(w + 0, hs->magic);
    w[4] = hs->version_major;
    w[5] = hs->version_minor;
    val_put_le16(w + 6, hs->reserved);
    val_put_le32(w + 8, hs->packet_size);
    val_put_le32(w + 12, hs->features);
    val_put_le32(w + 16, hs->required);
    val_put_le32(w + 20, hs->requested);
    val_put_le16(w + 24, hs->tx_max_window_packets);
    val_put_le16(w + 26, hs->rx_max_window_packets);
    w[28] = hs->ack_stride_packets;
    memcpy(w + 29, hs->reserved_capabilities, 3);
    val_put_le16(w + 32, hs->supported_features16);
    val_put_le16(w + 34, hs->required_features16);
    val_put_le16(w + 36, hs->requested_features16);
    w[38] = w[39] = 0; /* padding on the wire */
    val_put_le32(w + 40, hs->reserved2);
}

void val_deserialize_handshake(const uint8_t *wire_data, val_handshake_t *hs)
{
    if (!wire_data || !hs)
        return;
    const uint8_t *w = wire_data;
    hs->magic = val_get_le32(w + 0);
    hs->version_major = w[4];
    hs->version_minor = w[5];
    hs->reserved = val_get_le16(w + 6);
    hs->packet_size = val_get_le32(w + 8);
    hs->features = val_get_le32(w + 12);
    hs->required = val_get_le32(w + 16);
    hs->requested = val_get_le32(w + 20);
    hs->tx_max_window_packets = val_get_le16(w + 24);
    hs->rx_max_window_packets = val_get_le16(w + 26);
    hs->ack_stride_packets = w[28];
    memcpy(hs->reserved_capabilities, w + 29, 3);
    hs->supported_features16 = val_get_le16(w + 32);
    hs->required_features16 = val_get_le16(w + 34);
    hs->requested_features16 = val_get_le16(w + 36);
    hs->reserved2 = val_get_le32(w + 40);
}

#define VAL_META_NAME_BYTES (VAL_MAX_FILENAME + 1u)
#define VAL_META_PATH_BYTES (VAL_MAX_PATH + 1u)

void val_serialize_meta(const val_meta_payload_t *meta, uint8_t *wire_data)
{
    if (!meta || !wire_data)
        return;
    memcpy(wire_data, meta->filename, VAL_META_NAME_BYTES);
    memcpy(wire_data + VAL_META_NAME_BYTES, meta->sender_path, VAL_META_PATH_BYTES);
    val_put_le64(wire_data + VAL_META_NAME_BYTES + VAL_META_PATH_BYTES, meta->file_size);
}

void val_deserialize_meta(const uint8_t *wire_data, val_meta_payload_t *meta)
{
    if (!wire_data || !meta)
        return;
    memcpy(meta->filename, wire_data, VAL_META_NAME_BYTES);
    memcpy(meta->sender_path, wire_data + VAL_META_NAME_BYTES, VAL_META_PATH_BYTES);
    meta->file_size = val_get_le64(wire_data + VAL_META_NAME_BYTES + VAL_META_PATH_BYTES);
}

void val_serialize_resume_resp(const val_resume_resp_t *resp, uint8_t *wire_data)
{
    if (!resp || !wire_data)
        return;
    val_put_le32(wire_data, (uint32_t)resp->action);
    val_put_le64(wire_data + 4, resp->resume_offset);
    val_put_le32(wire_data + 12, resp->verify_crc);
    val_put_le64(wire_data + 16, resp->verify_length);
}

void val_deserialize_resume_resp(const uint8_t *wire_data, val_resume_resp_t *resp)
{
    if (!wire_data || !resp)
        return;
    resp->action = (val_resume_action_t)val_get_le32(wire_data);
    resp->resume_offset = val_get_le64(wire_data + 4);
    resp->verify_crc = val_get_le32(wire_data + 12);
    resp->verify_length = val_get_le64(wire_data + 16);
}

void val_serialize_verify_request(uint64_t offset, uint32_t crc, uint32_t length, uint8_t *wire_data)
{
    if (!wire_data)
        return;
    val_put_le64(wire_data, offset);
    val_put_le32(wire_data + 8, crc);
    val_put_le32(wire_data + 12, length);
}

void val_deserialize_verify_request(const uint8_t *wire_data, uint64_t *offset, uint32_t *crc, uint32_t *length)
{
    if (!wire_data)
        return;
    if (offset)
        *offset = val_get_le64(wire_data);
    if (crc)
        *crc = val_get_le32(wire_data + 8);
    if (length)
        *length = val_get_le32(wire_data + 12);
}

void val_serialize_verify_response(val_status_t result, uint32_t receiver_crc, uint8_t *wire_data)
{
    if (!wire_data)
        return;
    val_put_le32(wire_data, (uint32_t)result);
    val_put_le32(wire_data + 4, receiver_crc);
}

void val_deserialize_verify_response(const uint8_t *wire_data, val_status_t *result, uint32_t *receiver_crc)
{
    if (!wire_data)
        return;
    if (result)
        *result = (val_status_t)(int32_t)val_get_le32(wire_data);
    if (receiver_crc)
        *receiver_crc = val_get_le32(wire_data + 4);
}

void val_serialize_error_payload(const val_error_payload_t *payload, uint8_t *wire_data)
{
    if (!payload || !wire_data)
        return;
    val_put_le32(wire_data, (uint32_t)payload->code);
    val_put_le32(wire_data + 4, payload->detail);
}

void val_deserialize_error_payload(const uint8_t *wire_data, val_error_payload_t *payload)
{
    if (!wire_data || !payload)
        return;
    payload->code = (int32_t)val_get_le32(wire_data);
    payload->detail = val_get_le32(wire_data + 4);
}

/* ---- batch framing ------------------------------------------------------ */
val_status_t val_frame_data_batch(const uint8_t *payload, const uint64_t *pay_off, const uint32_t *pay_len,
                                  const uint64_t *file_off, const uint8_t *include_offset, uint32_t n, uint8_t *out,
                                  size_t out_cap, uint64_t *frame_off, uint32_t *crc_len, size_t *out_used)
{
    if (out_used)
        *out_used = 0;
    if (n && (!pay_len || !file_off || !out || !frame_off || !crc_len))
        return VAL_ERR_INVALID_ARG;
    size_t pos = 0;
    for (uint32_t i = 0; i < n; i++) {
        const int explicit_off = include_offset ? (include_offset[i] != 0) : 1;
        const uint64_t content = (uint64_t)pay_len[i] + (explicit_off ? 8u : 0u);
        if (content > VAL_WIRE_MAX_CONTENT)
            return VAL_ERR_INVALID_ARG; /* the reference would wrap content_len here */
        if (pay_len[i] && (!payload || !pay_off))
            return VAL_ERR_INVALID_ARG;
        const size_t wire = VAL_WIRE_HEADER_SIZE + (size_t)content + VAL_WIRE_TRAILER_SIZE;
        if (wire > out_cap - pos)
            return VAL_ERR_INVALID_ARG;
        uint8_t *f = out + pos;
        val_serialize_frame_header((uint8_t)VAL_PKT_DATA, explicit_off ? (uint8_t)VAL_DATA_OFFSET_PRESENT : 0u,
                                   (uint16_t)content, 0u, f);
        uint8_t *c = f + VAL_WIRE_HEADER_SIZE;
        if (explicit_off) {
            val_put_le64(c, file_off[i]);
            c += 8;
        }
        if (pay_len[i])
            memcpy(c, payload + pay_off[i], pay_len[i]);
        memset(f + VAL_WIRE_HEADER_SIZE + content, 0, VAL_WIRE_TRAILER_SIZE);
        frame_off[i] = pos;
        crc_len[i] = (uint32_t)(VAL_WIRE_HEADER_SIZE + content);
        pos += wire;
    }
    if (out_used)
        *out_used = pos;
    return VAL_OK;
}

void val_frame_put_trailers(uint8_t *stream, const uint64_t *frame_off, const uint32_t *crc_len, const uint32_t *crc,
                            uint32_t n)
{
    for (uint32_t i = 0; i < n; i++)
        val_put_le32(stream + frame_off[i] + crc_len[i], crc[i]);
}

val_status_t val_frame_scan(const uint8_t *stream, size_t len, size_t mtu, uint32_t max_frames, uint64_t *frame_off,
                            uint32_t *crc_len, uint32_t *n_frames, size_t *consumed)
{
    if (n_frames)
        *n_frames = 0;
    if (consumed)
        *consumed = 0;
    if ((!stream && len) || !frame_off || !crc_len)
        return VAL_ERR_INVALID_ARG;
    if (mtu < VAL_WIRE_HEADER_SIZE + VAL_WIRE_TRAILER_SIZE)
        return VAL_ERR_INVALID_ARG;
    const size_t max_content = mtu - VAL_WIRE_HEADER_SIZE - VAL_WIRE_TRAILER_SIZE;
    size_t pos = 0;
    uint32_t k = 0;
    val_status_t st = VAL_OK;
    while (k < max_frames && len - pos >= VAL_WIRE_HEADER_SIZE) {
        uint16_t content = 0;
        val_deserialize_frame_header(stream + pos, NULL, NULL, &content, NULL);
        if ((size_t)content > max_content) {
            st = VAL_ERR_PROTOCOL;
            break;
        }
        const size_t wire = VAL_WIRE_HEADER_SIZE + (size_t)content + VAL_WIRE_TRAILER_SIZE;
        if (len - pos < wire)
            break; /* incomplete frame: wait for more bytes */
        frame_off[k] = pos;
        crc_len[k] = (uint32_t)(VAL_WIRE_HEADER_SIZE + content);
        k++;
        pos += wire;
    }
    if (n_frames)
        *n_frames = k;
    if (consumed)
        *consumed = pos;
    return st;
}

void val_frame_payload_lens(const uint8_t *stream, const uint64_t *frame_off, const uint32_t *crc_len, uint32_t n,
                            uint32_t *pay_len)
{
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t L = crc_len[i];
        uint32_t pre = VAL_WIRE_HEADER_SIZE;
        if (L >= VAL_WIRE_HEADER_SIZE && (stream[frame_off[i] + 1] & VAL_DATA_OFFSET_PRESENT))
            pre += 8u;
        pay_len[i] = L >= pre ? L - pre : 0u;
    }
}

void val_frame_data_offsets(const uint8_t *stream, const uint64_t *frame_off, const uint32_t *crc_len, uint32_t n,
                            uint64_t *file_off)
{
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t *f = stream + frame_off[i];
        const uint32_t L = crc_len[i];
        if (L < VAL_WIRE_HEADER_SIZE || f[0] != (uint8_t)VAL_PKT_DATA)
            file_off[i] = VAL_FRAME_OFFSET_NOT_DATA;
        else if (!(f[1] & VAL_DATA_OFFSET_PRESENT))
            file_off[i] = VAL_FRAME_OFFSET_IMPLIED;
        else if (L < VAL_WIRE_HEADER_SIZE + 8u)
            file_off[i] = VAL_FRAME_OFFSET_NOT_DATA; /* no room for the offset: never folded */
        else
            file_off[i] = val_get_le64(f + VAL_WIRE_HEADER_SIZE);
    }
}
