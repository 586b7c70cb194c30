/*
 * val_errors.h -- status codes and CRC error-detail bits used by the
 * MI355X CRC-32 integrity path. Numeric values are wire/ABI compatible with
 * VAL v0.7 (reference include/val_errors.h:18-39 status enum,
 * :77-80 CRC detail bits).
 */
#ifndef VAL_ERRORS_H
#define VAL_ERRORS_H
#include <stdint.h>

typedef enum {
    VAL_OK = 0,
    VAL_SKIPPED = 1,
    VAL_ERR_INVALID_ARG = -1,   /* bad descriptor, NULL pointer, frame overruns buffer */
    VAL_ERR_NO_MEMORY = -2,     /* device or pinned allocation failed */
    VAL_ERR_IO = -3,            /* HIP runtime/device failure */
    VAL_ERR_TIMEOUT = -4,
    VAL_ERR_PROTOCOL = -5,
    VAL_ERR_CRC = -6,           /* one or more trailer CRC mismatches */
    VAL_ERR_RESUME_VERIFY = -7,
    VAL_ERR_INCOMPATIBLE_VERSION = -8,
    VAL_ERR_PACKET_SIZE_MISMATCH = -9,
    VAL_ERR_FEATURE_NEGOTIATION = -10,
    VAL_ERR_ABORTED = -11,
    VAL_ERR_MODE_NEGOTIATION_FAILED = -12,
    VAL_ERR_UNSUPPORTED_TX_MODE = -14,
    VAL_ERR_PERFORMANCE = -15
} val_status_t;

/* CRC category of the 32-bit error-detail mask. */
#define VAL_ERROR_DETAIL_CRC_HEADER     ((uint32_t)0x00000100) /* header_crc mismatch (defined by this build) */
#define VAL_ERROR_DETAIL_CRC_TRAILER    ((uint32_t)0x00000200) /* trailer CRC mismatch */
#define VAL_ERROR_DETAIL_CRC_RESUME     ((uint32_t)0x00000800) /* resume verify-window mismatch */
#define VAL_ERROR_DETAIL_SIZE_MISMATCH  ((uint32_t)0x00001000)
#define VAL_ERROR_DETAIL_PACKET_CORRUPT ((uint32_t)0x00002000)
#define VAL_ERROR_DETAIL_PAYLOAD_SIZE   ((uint32_t)0x00020000) /* content_len beyond MTU / 16-bit field */

#endif /* VAL_ERRORS_H */
