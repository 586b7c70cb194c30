/*
 * val_protocol.h -- public surface of VAL v0.7 that the MI355X CRC-32
 * integrity path plugs into.
 *
 * Scope: this build replaces the per-frame CRC engine behind VAL's
 * `crc32_provider` hook and the `val_crc32*` functions. It keeps the
 * reference's type names, constants and struct layouts so that a VAL sender
 * or receiver built against the reference headers can install
 * `val_gpu_crc32_provider` (val_crc32_gpu.h) unchanged:
 *   - crc32_func_t                reference include/val_protocol.h:163-166
 *   - val_config_t.crc32_provider reference include/val_protocol.h:264-266
 *     (byte offset 96, sizeof(val_config_t) == 312 on LP64; pinned by
 *      tests/test_abi.py against the reference's own layout)
 *   - val_crc32                   reference include/val_protocol.h:377
 * Session, transport, filesystem and flow-control *behaviour* stays in the
 * reference's control plane. Its public surface is declared here unchanged
 * (types, constants, the session API of reference :363-446), so the
 * reference's own src/val_core.c, val_sender.c, val_receiver.c and
 * val_wire.c compile against these headers (tests/test_header_surface.py)
 * and link against this library's val_crc32* / provider.
 */
#ifndef VAL_PROTOCOL_H
#define VAL_PROTOCOL_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#include "val_byte_order.h"
#include "val_errors.h"

#ifdef __cplusplus
extern "C" {
#endif

#define VAL_MAGIC 0x56414C00u /* "VAL\0" */
#define VAL_VERSION_MAJOR 0u
#define VAL_VERSION_MINOR 7u
#define VAL_MIN_PACKET_SIZE 512u
#define VAL_MAX_PACKET_SIZE (2u * 1024u * 1024u)
#define VAL_MAX_FILENAME 127u
#define VAL_MAX_PATH 127u
#define VAL_PKT_CANCEL 0x18u

typedef enum {
    VAL_PKT_HELLO = 1,
    VAL_PKT_SEND_META = 2,
    VAL_PKT_RESUME_REQ = 3,
    VAL_PKT_RESUME_RESP = 4,
    VAL_PKT_DATA = 5,
    VAL_PKT_DATA_ACK = 6,
    VAL_PKT_VERIFY = 7,
    VAL_PKT_DONE = 8,
    VAL_PKT_ERROR = 9,
    VAL_PKT_EOT = 10,
    VAL_PKT_EOT_ACK = 11,
    VAL_PKT_DONE_ACK = 12,
    VAL_PKT_DATA_NAK = 13
} val_packet_type_t;

/* DATA_ACK payload flags (reserved by v0.7) */
typedef enum { VAL_ACK_FLAG_HEARTBEAT = 1u << 0, VAL_ACK_FLAG_EOF = 1u << 1 } val_ack_flags_t;

/*
 * CRC-32 provider hook. Semantics fixed by the reference's call sites
 * (src/val_core.c:399-406, :431-438), which always pass seed = 0xFFFFFFFF and
 * expect the finished CRC:  provider(seed, buf, len) ==
 * val_crc32_finalize_state(val_crc32_update_state(seed, buf, len)).
 */
typedef uint32_t (*crc32_func_t)(uint32_t seed, const void *buf, size_t len);

/* One on-wire packet as seen by the capture hook. */
typedef enum { VAL_DIR_TX = 1, VAL_DIR_RX = 2 } val_packet_direction_t;
typedef struct val_packet_record_t {
    val_packet_direction_t direction;
    uint8_t type;
    uint32_t wire_len;    /* header + content + trailer */
    uint32_t payload_len;
    uint64_t offset;
    bool crc_ok;          /* RX: trailer verified */
    uint32_t timestamp_ms;
    const void *session_id;
} val_packet_record_t;

typedef struct val_session_s val_session_t;

typedef struct {
    void *(*alloc)(size_t size, void *context);
    void (*free)(void *ptr, void *context);
    void *context;
} val_memory_allocator_t;

typedef enum { VAL_RESUME_NEVER = 0, VAL_RESUME_SKIP_EXISTING = 1, VAL_RESUME_TAIL = 2 } val_resume_mode_t;

/* Receiver's answer to RESUME_REQ (wire form: val_serialize_resume_resp). */
typedef enum {
    VAL_RESUME_START_ZERO = 0,
    VAL_RESUME_START_OFFSET = 1,
    VAL_RESUME_VERIFY_FIRST = 2,
    VAL_RESUME_SKIP_FILE = 3,
    VAL_RESUME_ABORT_FILE = 4
} val_resume_action_t;

typedef struct {
    val_resume_action_t action;
    uint64_t resume_offset;
    uint32_t verify_crc;    /* CRC-32 of the verify window: the region CRC (val_crc32_region_dev) */
    uint64_t verify_length;
} val_resume_resp_t;

typedef enum {
    VAL_LOG_OFF = 0,
    VAL_LOG_CRITICAL = 1,
    VAL_LOG_WARNING = 2,
    VAL_LOG_INFO = 3,
    VAL_LOG_DEBUG = 4,
    VAL_LOG_TRACE = 5
} val_log_level_t;

/* Optional features negotiated in the handshake: none are defined in v0.7. */
#define VAL_FEAT_NONE 0u
#define VAL_BUILTIN_FEATURES VAL_FEAT_NONE

typedef struct {
    val_resume_mode_t mode;
    uint32_t tail_cap_bytes;   /* TAIL verify window cap; reference clamps to 256 MiB */
    uint32_t min_verify_bytes;
    bool mismatch_skip;
    uint8_t reserved0;
    uint16_t reserved1;
} val_resume_config_t;

typedef struct {
    uint16_t window_cap_packets;  /* max frames in flight: the natural batch size for the GPU path */
    uint16_t initial_cwnd_packets;
    bool retransmit_cache_enabled;
    uint8_t reserved0;
    uint16_t degrade_error_threshold;
    uint16_t recovery_success_threshold;
    val_memory_allocator_t allocator;
} val_tx_flow_config_t;

typedef struct val_meta_payload_t {
    char filename[VAL_MAX_FILENAME + 1];
    char sender_path[VAL_MAX_PATH + 1];
    uint64_t file_size;
} val_meta_payload_t;

typedef struct {
    uint64_t bytes_transferred;
    uint64_t total_bytes;
    uint64_t current_file_bytes;
    uint32_t files_completed;
    uint32_t total_files;
    uint32_t transfer_rate_bps;
    uint32_t eta_seconds;
    const char *current_filename;
} val_progress_info_t;

typedef enum { VAL_VALIDATION_ACCEPT = 0, VAL_VALIDATION_SKIP = 1, VAL_VALIDATION_ABORT = 2 } val_validation_action_t;
typedef val_validation_action_t (*val_metadata_validator_t)(const val_meta_payload_t *meta, const char *target_path,
                                                            void *context);

/* Session configuration: layout-identical to the reference (see header note). */
typedef struct {
    struct {
        int (*send)(void *ctx, const void *data, size_t len);
        int (*recv)(void *ctx, void *buffer, size_t buffer_size, size_t *received, uint32_t timeout_ms);
        int (*is_connected)(void *ctx);
        void (*flush)(void *ctx);
        void *io_context;
    } transport;
    struct {
        void *(*fopen)(void *ctx, const char *path, const char *mode);
        size_t (*fread)(void *ctx, void *buffer, size_t size, size_t count, void *file);
        size_t (*fwrite)(void *ctx, const void *buffer, size_t size, size_t count, void *file);
        int (*fseek)(void *ctx, void *file, int64_t offset, int whence);
        int64_t (*ftell)(void *ctx, void *file);
        int (*fclose)(void *ctx, void *file);
        void *fs_context;
    } filesystem;
    crc32_func_t crc32_provider; /* NULL = built-in software CRC; set to val_gpu_crc32_provider */
    struct {
        uint32_t (*get_ticks_ms)(void);
        void (*delay_ms)(uint32_t ms);
    } system;
    struct {
        uint32_t min_timeout_ms;
        uint32_t max_timeout_ms;
        uint32_t handshake_budget_ms;
    } timeouts;
    struct {
        uint32_t required;
        uint32_t requested;
    } features;
    struct {
        uint8_t meta_retries;
        uint8_t data_retries;
        uint8_t ack_retries;
        uint8_t handshake_retries;
        uint32_t backoff_ms_base;
    } retries;
    struct {
        void *send_buffer;  /* >= packet_size bytes: header + content + trailer staging */
        void *recv_buffer;
        size_t packet_size; /* MTU */
    } buffers;
    val_resume_config_t resume;
    val_tx_flow_config_t tx_flow;
    struct {
        void (*on_file_start)(const char *filename, const char *sender_path, uint64_t file_size, uint64_t resume_offset);
        void (*on_file_complete)(const char *filename, const char *sender_path, val_status_t result);
        void (*on_progress)(const val_progress_info_t *info);
    } callbacks;
    struct {
        val_metadata_validator_t validator;
        void *validator_context;
    } metadata_validation;
    struct {
        void (*log)(void *ctx, int level, const char *file, int line, const char *message);
        void *context;
        int min_level;
    } debug;
    struct {
        void (*on_packet)(void *ctx, const val_packet_record_t *rec);
        void *context;
    } capture;
} val_config_t;

/* ---- session API (implemented by the reference's control plane, which
 * this library does not replace; declared so its sources build here) ---- */
/* control-plane API begin */
val_status_t val_session_create(const val_config_t *config, val_session_t **out_session, uint32_t *out_detail);
void val_session_destroy(val_session_t *session);
val_status_t val_send_files(val_session_t *session, const char *const *filepaths, size_t file_count,
                            const char *sender_path);
val_status_t val_receive_files(val_session_t *session, const char *output_directory);
void val_clean_filename(const char *input, char *output, size_t output_size);
void val_clean_path(const char *input, char *output, size_t output_size);
val_status_t val_get_cwnd_packets(val_session_t *session, uint32_t *out_cwnd);
val_status_t val_get_peer_tx_cap_packets(val_session_t *session, uint32_t *out_cap);
val_status_t val_get_effective_packet_size(val_session_t *session, size_t *out_packet_size);
uint32_t val_get_builtin_features(void);
val_status_t val_get_last_error(val_session_t *session, val_status_t *code, uint32_t *detail_mask);
val_status_t val_get_error(val_session_t *session, val_error_t *out);
val_status_t val_emergency_cancel(val_session_t *session);
bool val_check_for_cancel(val_session_t *session);
void val_config_validation_disabled(val_config_t *config);
void val_config_set_validator(val_config_t *config, val_metadata_validator_t validator, void *context);

#if VAL_ENABLE_METRICS
/* Per-session counters (reference builds with VAL_ENABLE_METRICS=1);
 * crc_errors is what val_crc32_verify_frames_* count per batch. */
typedef struct {
    uint64_t packets_sent;
    uint64_t packets_recv;
    uint64_t bytes_sent;
    uint64_t bytes_recv;
    uint64_t send_by_type[32]; /* by on-wire type byte, CANCEL (0x18) included */
    uint64_t recv_by_type[32];
    uint32_t timeouts;
    uint32_t timeouts_hard;
    uint32_t retransmits;
    uint32_t crc_errors;
    uint32_t handshakes;
    uint32_t files_sent;
    uint32_t files_recv;
    uint32_t rtt_samples;
} val_metrics_t;
val_status_t val_get_metrics(val_session_t *session, val_metrics_t *out);
val_status_t val_reset_metrics(val_session_t *session);
#endif
/* control-plane API end */

/* ---- CRC-32/ISO-HDLC (reflected poly 0xEDB88320, init and xorout
 * 0xFFFFFFFF): implemented by this library (val_crc32_gpu.h has the batch
 * forms and the provider). val_crc32 is the reference's public utility
 * (:377); the state functions are its internal incremental API
 * (src/val_internal.h:628-641). */
uint32_t val_crc32(const void *data, size_t length);
uint32_t val_crc32_init_state(void);
uint32_t val_crc32_update_state(uint32_t state, const void *data, size_t length);
uint32_t val_crc32_finalize_state(uint32_t state);

#ifdef __cplusplus
}
#endif
#endif /* VAL_PROTOCOL_H */
