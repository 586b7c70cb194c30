/*
 * gen_golden.c -- emits golden vectors from the REFERENCE library itself.
 * TEST INFRASTRUCTURE; runs only in the build container (needs
 * /root/reference). Links oracle/_ref objects compiled from
 * /root/reference/src (see oracle/Makefile) and calls:
 *   val_crc32                       src/val_core.c:150
 *   val_crc32_{init,update,finalize}_state   src/val_core.c:162-183
 *   val_internal_send_packet_ex     src/val_core.c:874 (TX framing + trailer)
 * Output: JSON on stdout (tests/golden/ref_vectors.json).
 */
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "val_protocol.h"
#include "val_internal.h"
#include "val_wire.h"
#include "prng.h"

static uint8_t *g_cap;
static size_t g_cap_len;
static int cap_send(void *ctx, const void *data, size_t len)
{
    (void)ctx;
    memcpy(g_cap, data, len);
    g_cap_len = len;
    return (int)len;
}
static int cap_recv(void *ctx, void *b, size_t n, size_t *got, uint32_t t)
{
    (void)ctx; (void)b; (void)n; (void)t;
    if (got) *got = 0;
    return -1;
}
static uint32_t ticks(void) { return 0; }
static void delay(uint32_t ms) { (void)ms; }

static void hexdump(const uint8_t *p, size_t n)
{
    printf("\"");
    for (size_t i = 0; i < n; i++) printf("%02x", p[i]);
    printf("\"");
}

int main(void)
{
    const size_t MAXN = 16u << 20;
    uint8_t *buf = (uint8_t *)malloc(MAXN);
    printf("{\n");
    printf("  \"generator\": \"oracle/gen_golden.c linked against /root/reference/src (VAL v0.7.0)\",\n");
    printf("  \"prng\": \"byte i of stream s = LE byte (i%%8) of splitmix64(s + (i/8+1)*0x9E3779B97F4A7C15)\",\n");

    /* F1 KATs */
    printf("  \"kat_123456789\": %u,\n", val_crc32("123456789", 9));
    printf("  \"kat_empty\": %u,\n", val_crc32("", 0));
    printf("  \"single_bytes\": [");
    for (int b = 0; b < 256; b++) {
        uint8_t v = (uint8_t)b;
        printf("%s%u", b ? "," : "", val_crc32(&v, 1));
    }
    printf("],\n");

    /* F2 length sweep over stream 0xF2 prefixes */
    oracle_prng_fill(0xF2u, buf, 70000);
    printf("  \"sweep_seed\": %u,\n  \"sweep_0_4096\": [", 0xF2u);
    for (int L = 0; L <= 4096; L++) printf("%s%u", L ? "," : "", val_crc32(buf, (size_t)L));
    printf("],\n");
    const size_t special[] = {1020, 1040, 16400, 65524, 65532, 65535, 65543};
    printf("  \"sweep_special\": {");
    for (size_t i = 0; i < sizeof(special) / sizeof(special[0]); i++)
        printf("%s\"%zu\": %u", i ? ", " : "", special[i], val_crc32(buf, special[i]));
    printf("},\n");

    /* provider semantics: seeds other than 0xFFFFFFFF via raw state API */
    printf("  \"state_vectors\": [");
    const uint32_t seeds[] = {0xFFFFFFFFu, 0u, 0x12345678u, 0xDEADBEEFu};
    const size_t lens[] = {0, 1, 3, 4, 7, 8, 100, 1040};
    int first = 1;
    for (size_t s = 0; s < 4; s++)
        for (size_t l = 0; l < sizeof(lens) / sizeof(lens[0]); l++) {
            uint32_t st = val_crc32_update_state(seeds[s], buf, lens[l]);
            printf("%s{\"seed\": %u, \"len\": %zu, \"state\": %u, \"final\": %u}", first ? "" : ",", seeds[s], lens[l], st,
                   val_crc32_finalize_state(st));
            first = 0;
        }
    printf("],\n");

    /* F4 incremental == one-shot; region windows over stream 0xF4 */
    oracle_prng_fill(0xF4u, buf, 8u << 20);
    const size_t windows[] = {1024, 8192, 65536, 8u << 20};
    const size_t chunks[] = {512, 1024, 2048, 65536};
    printf("  \"region_seed\": %u,\n  \"regions\": [", 0xF4u);
    first = 1;
    for (size_t w = 0; w < 4; w++)
        for (size_t c = 0; c < 4; c++) {
            uint32_t st = val_crc32_init_state();
            for (size_t o = 0; o < windows[w]; o += chunks[c]) {
                size_t take = windows[w] - o < chunks[c] ? windows[w] - o : chunks[c];
                st = val_crc32_update_state(st, buf + o, take);
            }
            printf("%s{\"len\": %zu, \"chunk\": %zu, \"crc\": %u, \"oneshot\": %u}", first ? "" : ",", windows[w], chunks[c],
                   val_crc32_finalize_state(st), val_crc32(buf, windows[w]));
            first = 0;
        }
    printf("],\n");

    /* F5 combine triples: A = stream 0xF5 [0,la), B = next lb bytes */
    oracle_prng_fill(0xF5u, buf, 300000);
    const size_t la_[] = {0, 1, 7, 1040, 16400, 65532, 100000};
    const size_t lb_[] = {0, 1, 5, 1024, 16400, 65536, 131072};
    printf("  \"combine_seed\": %u,\n  \"combine\": [", 0xF5u);
    first = 1;
    for (size_t a = 0; a < 7; a++)
        for (size_t b = 0; b < 7; b++) {
            printf("%s[%zu,%zu,%u,%u,%u]", first ? "" : ",", la_[a], lb_[b], val_crc32(buf, la_[a]),
                   val_crc32(buf + la_[a], lb_[b]), val_crc32(buf, la_[a] + lb_[b]));
            first = 0;
        }
    printf("],\n");

    /* F3 frames via the reference TX path */
    size_t P = VAL_MAX_PACKET_SIZE;
    uint8_t *sb = (uint8_t *)calloc(1, P), *rb = (uint8_t *)calloc(1, P);
    g_cap = (uint8_t *)malloc(P + 64);
    val_config_t cfg;
    memset(&cfg, 0, sizeof(cfg));
    cfg.transport.send = cap_send;
    cfg.transport.recv = cap_recv;
    cfg.system.get_ticks_ms = ticks;
    cfg.system.delay_ms = delay;
    cfg.buffers.send_buffer = sb;
    cfg.buffers.recv_buffer = rb;
    cfg.buffers.packet_size = P;
    cfg.timeouts.min_timeout_ms = 10;
    cfg.timeouts.max_timeout_ms = 100;
    val_session_t *s = NULL;
    if (val_session_create(&cfg, &s, NULL) != VAL_OK) {
        fprintf(stderr, "session create failed\n");
        return 1;
    }
    const uint32_t payloads[] = {0, 1, 492, 1004, 1024, 16384, 65516, 65527, 65528, 65536};
    const uint64_t offs[] = {0ull, (1ull << 32) + 5u};
    printf("  \"frames_payload_seed_base\": %u,\n  \"frames\": [", 0xF3u);
    first = 1;
    uint8_t *pl = (uint8_t *)malloc(70000);
    for (size_t pi = 0; pi < sizeof(payloads) / sizeof(payloads[0]); pi++)
        for (size_t oi = 0; oi < 2; oi++)
            for (int inc = 0; inc <= 1; inc++) {
                uint64_t seed = 0xF3u ^ ((uint64_t)payloads[pi] << 8);
                oracle_prng_fill(seed, pl, payloads[pi]);
                g_cap_len = 0;
                int rc = val_internal_send_packet_ex(s, VAL_PKT_DATA, pl, payloads[pi], offs[oi], inc);
                size_t w = g_cap_len;
                printf("%s{\"payload_len\": %u, \"offset\": %llu, \"include_offset\": %d, \"rc\": %d, \"wire_len\": %zu, ", first ? "" : ",",
                       payloads[pi], (unsigned long long)offs[oi], inc, rc, w);
                printf("\"header\": ");
                hexdump(g_cap, w >= 8 ? 8 : w);
                printf(", \"trailer\": ");
                hexdump(g_cap + (w >= 4 ? w - 4 : 0), w >= 4 ? 4 : 0);
                printf(", \"crc_input_crc\": %u", w >= 4 ? val_crc32(g_cap, w - 4) : 0u);
                if (w <= 1100) {
                    printf(", \"wire\": ");
                    hexdump(g_cap, w);
                }
                printf("}");
                first = 0;
            }
    printf("],\n");
    val_session_destroy(s);

    /* F7 ABI layout of the public surface the drop-in keeps */
    printf("  \"abi\": {\"sizeof_val_config_t\": %zu, \"offsetof_crc32_provider\": %zu, \"sizeof_val_packet_record_t\": %zu, "
           "\"sizeof_val_handshake_t\": %zu, \"offsetof_buffers\": %zu}\n",
           sizeof(val_config_t), offsetof(val_config_t, crc32_provider), sizeof(val_packet_record_t), sizeof(val_handshake_t),
           offsetof(val_config_t, buffers));
    printf("}\n");
    return 0;
}
