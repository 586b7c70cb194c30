/*
 * val_errors.h -- VAL v0.7 status codes and the 32-bit error-detail mask,
 * numerically identical to the reference (include/val_errors.h:18-135), so a
 * VAL sender or receiver compiled against these headers behaves the same.
 * Statuses the MI355X CRC path itself returns: VAL_OK, VAL_ERR_INVALID_ARG
 * (bad descriptor, NULL pointer, frame overruns its buffer), VAL_ERR_NO_MEMORY
 * (device or pinned allocation), VAL_ERR_IO (HIP runtime or device failure),
 * VAL_ERR_PROTOCOL (frame scan: content beyond the MTU) and VAL_ERR_CRC (one
 * or more trailer mismatches in a verify batch).
 */
#ifndef VAL_ERRORS_H
#define VAL_ERRORS_H
#include <stdint.h>

typedef enum {
    VAL_OK = 0,
    VAL_SKIPPED = 1, /* informational: a file was skipped */
    VAL_ERR_INVALID_ARG = -1,
    VAL_ERR_NO_MEMORY = -2,
    VAL_ERR_IO = -3,
    VAL_ERR_TIMEOUT = -4,
    VAL_ERR_PROTOCOL = -5,
    VAL_ERR_CRC = -6,
    VAL_ERR_RESUME_VERIFY = -7,
    VAL_ERR_INCOMPATIBLE_VERSION = -8,
    VAL_ERR_PACKET_SIZE_MISMATCH = -9,
    VAL_ERR_FEATURE_NEGOTIATION = -10,
    VAL_ERR_ABORTED = -11,
    VAL_ERR_MODE_NEGOTIATION_FAILED = -12,
    VAL_ERR_UNSUPPORTED_TX_MODE = -14,
    VAL_ERR_PERFORMANCE = -15
} val_status_t;

/* Status plus detail mask and an optional static site name (never freed). */
typedef struct {
    val_status_t code;
    uint32_t detail;
    const char *op;
} val_error_t;

/* Detail mask: bits 0-7 network, 8-15 CRC/integrity, 16-23 protocol,
 * 24-27 filesystem, 28-31 context selector. */
#define VAL_ERROR_DETAIL_NET_MASK ((uint32_t)0x000000FFu)
#define VAL_ERROR_DETAIL_CRC_MASK ((uint32_t)0x0000FF00u)
#define VAL_ERROR_DETAIL_PROTO_MASK ((uint32_t)0x00FF0000u)
#define VAL_ERROR_DETAIL_FS_MASK ((uint32_t)0x0F000000u)
#define VAL_ERROR_DETAIL_CONTEXT_MASK ((uint32_t)0xF0000000u)

/* network */
#define VAL_ERROR_DETAIL_NETWORK_RESET ((uint32_t)0x00000001u)
#define VAL_ERROR_DETAIL_TIMEOUT_ACK ((uint32_t)0x00000002u)
#define VAL_ERROR_DETAIL_TIMEOUT_DATA ((uint32_t)0x00000004u)
#define VAL_ERROR_DETAIL_TIMEOUT_META ((uint32_t)0x00000008u)
#define VAL_ERROR_DETAIL_TIMEOUT_HELLO ((uint32_t)0x00000010u)
#define VAL_ERROR_DETAIL_SEND_FAILED ((uint32_t)0x00000020u)
#define VAL_ERROR_DETAIL_RECV_FAILED ((uint32_t)0x00000040u)
#define VAL_ERROR_DETAIL_CONNECTION ((uint32_t)0x00000080u)

/* CRC / integrity (CRC_HEADER: this build's header_crc) */
#define VAL_ERROR_DETAIL_CRC_HEADER ((uint32_t)0x00000100u)
#define VAL_ERROR_DETAIL_CRC_TRAILER ((uint32_t)0x00000200u)
#define VAL_ERROR_DETAIL_CRC_RESUME ((uint32_t)0x00000800u)
#define VAL_ERROR_DETAIL_SIZE_MISMATCH ((uint32_t)0x00001000u)
#define VAL_ERROR_DETAIL_PACKET_CORRUPT ((uint32_t)0x00002000u)
#define VAL_ERROR_DETAIL_SEQ_ERROR ((uint32_t)0x00004000u)
#define VAL_ERROR_DETAIL_OFFSET_ERROR ((uint32_t)0x00008000u)

/* protocol / features */
#define VAL_ERROR_DETAIL_VERSION ((uint32_t)0x00010000u)
#define VAL_ERROR_DETAIL_PACKET_SIZE ((uint32_t)0x00020000u)
#define VAL_ERROR_DETAIL_FEATURE_MISSING ((uint32_t)0x00040000u)
#define VAL_ERROR_DETAIL_INVALID_STATE ((uint32_t)0x00080000u)
#define VAL_ERROR_DETAIL_MALFORMED_PKT ((uint32_t)0x00100000u)
#define VAL_ERROR_DETAIL_UNKNOWN_TYPE ((uint32_t)0x00200000u)
#define VAL_ERROR_DETAIL_PAYLOAD_SIZE ((uint32_t)0x00400000u)
#define VAL_ERROR_DETAIL_EXCESSIVE_RETRIES ((uint32_t)0x00800000u)

/* filesystem */
#define VAL_ERROR_DETAIL_FILE_NOT_FOUND ((uint32_t)0x01000000u)
#define VAL_ERROR_DETAIL_FILE_LOCKED ((uint32_t)0x02000000u)
#define VAL_ERROR_DETAIL_DISK_FULL ((uint32_t)0x04000000u)
#define VAL_ERROR_DETAIL_PERMISSION ((uint32_t)0x08000000u)

/* context selector in bits 28-31 */
#define VAL_ERROR_CONTEXT_SHIFT 28
#define VAL_ERROR_CONTEXT_NONE 0u
#define VAL_ERROR_CONTEXT_MISSING_FEATURES 1u
#define VAL_ERROR_CONTEXT_MISSING_HOOKS 2u
#define VAL_ERROR_CONTEXT(detail) (((uint32_t)(detail)&VAL_ERROR_DETAIL_CONTEXT_MASK) >> VAL_ERROR_CONTEXT_SHIFT)

/* missing features: context 1, feature bits in the low 24, FEATURE_MISSING set */
#define VAL_SET_MISSING_FEATURE(mask)                                                                           \
    (((uint32_t)VAL_ERROR_CONTEXT_MISSING_FEATURES << VAL_ERROR_CONTEXT_SHIFT) | ((uint32_t)(mask)&0x00FFFFFFu) | \
     VAL_ERROR_DETAIL_FEATURE_MISSING)
#define VAL_GET_MISSING_FEATURE(detail)                                                                         \
    ((VAL_ERROR_CONTEXT(detail) == VAL_ERROR_CONTEXT_MISSING_FEATURES)                                          \
         ? (((detail)&0x00FFFFFFu) & ~VAL_ERROR_DETAIL_PROTO_MASK)                                              \
         : 0u)
/* missing required hooks: context 2 plus INVALID_STATE */
#define VAL_SET_MISSING_HOOKS() \
    (((uint32_t)VAL_ERROR_CONTEXT_MISSING_HOOKS << VAL_ERROR_CONTEXT_SHIFT) | VAL_ERROR_DETAIL_INVALID_STATE)
#define VAL_ERROR_IS_MISSING_HOOKS(detail) (VAL_ERROR_CONTEXT(detail) == VAL_ERROR_CONTEXT_MISSING_HOOKS)

#define VAL_ERROR_IS_NETWORK_RELATED(detail) (((detail)&VAL_ERROR_DETAIL_NET_MASK) != 0)
#define VAL_ERROR_IS_CRC_RELATED(detail) (((detail)&VAL_ERROR_DETAIL_CRC_MASK) != 0)
#define VAL_ERROR_IS_PROTOCOL_RELATED(detail) (((detail)&VAL_ERROR_DETAIL_PROTO_MASK) != 0)
#define VAL_ERROR_IS_FILESYSTEM_RELATED(detail) (((detail)&VAL_ERROR_DETAIL_FS_MASK) != 0)

#endif /* VAL_ERRORS_H */
