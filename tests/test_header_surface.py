"""The drop-in header surface (north_star: "keeping the
include/val_protocol.h and include/val_wire.h surface so it drops in under
src/val_sender.c and src/val_receiver.c").

Always (CPU, no GPU):
  * val_handshake_t and the other control payloads have the reference's wire
    sizes (golden abi block: sizeof_val_handshake_t 44, measured on the
    reference headers);
  * this library's control codecs reproduce, byte for byte, the HELLO /
    SEND_META / RESUME_RESP frames of the reference's own 1 MiB loopback
    transfer (tests/golden/dropin_vectors.json, F6).
Where the reference tree is present (the build container only):
  * every struct layout, enum value and object-like VAL_* macro of the
    reference's public headers equals ours;
  * the reference's src/val_core.c, val_sender.c, val_receiver.c and
    val_wire.c compile against include/ (not the reference's headers);
  * the reference's protocol code built against include/ regenerates both
    golden fixture files byte for byte;
  * the reference's src/val_wire.c codecs, compiled against include/, write
    the same bytes as this library's codecs for random payloads.
"""
import ctypes
import json
import os
import re
import shutil
import struct
import subprocess
import tempfile

import pytest

import val_protocol_amd.crc as vc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")
REF = "/root/reference"
HAVE_REF = os.path.isdir(os.path.join(REF, "src")) and os.path.isdir(os.path.join(REF, "include"))
REF_SRCS = [os.path.join(REF, "src", f) for f in ("val_core.c", "val_wire.c", "val_sender.c", "val_receiver.c")]
needs_gcc = pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
needs_ref = pytest.mark.skipif(not HAVE_REF, reason="reference tree absent (build container only)")


def _gcc(args, cwd=None):
    r = subprocess.run(["gcc", *args], capture_output=True, text=True, cwd=cwd)
    assert r.returncode == 0, r.stderr[-4000:]
    return r


def _run(exe, *args):
    return subprocess.run([exe, *args], check=True, capture_output=True, text=True, timeout=120).stdout


# ---- always ---------------------------------------------------------------
@needs_gcc
def test_control_payload_sizes(golden):
    src = r"""
    #include <stdio.h>
    #include <stddef.h>
    #include "val_wire.h"
    int main(void) {
        printf("%zu %zu %zu %u %u %u %u %u %u %zu\n", sizeof(val_handshake_t), sizeof(val_error_payload_t),
               offsetof(val_handshake_t, reserved2), VAL_WIRE_HANDSHAKE_SIZE, VAL_WIRE_META_SIZE,
               VAL_WIRE_RESUME_RESP_SIZE, VAL_WIRE_VERIFY_REQ_SIZE, VAL_WIRE_VERIFY_RESP_SIZE,
               VAL_WIRE_ERROR_PAYLOAD_SIZE, sizeof(val_meta_payload_t));
        return 0;
    }
    """
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "t.c"), "w").write(src)
        _gcc(["-std=c99", "-Wall", "-Werror", f"-I{INC}", "t.c", "-o", "t"], cwd=d)
        got = [int(x) for x in _run(os.path.join(d, "t")).split()]
    assert got[0] == golden["abi"]["sizeof_val_handshake_t"] == 44
    assert got[1:] == [8, 40, 44, 264, 24, 16, 8, 8, 264]


def _ctrl_frames(kind):
    lb = json.load(open(os.path.join(ROOT, "tests", "golden", "dropin_vectors.json")))["loopback"]
    return [bytes.fromhex(f[4]) for f in lb["tx_frames"] + lb["rx_frames"] if f[0] == kind]


def test_codecs_reproduce_reference_control_frames():
    lib = vc.lib()
    hello = _ctrl_frames(1)
    assert hello, "fixture holds HELLO frames"
    hs = ctypes.create_string_buffer(64)  # val_handshake_t (44 B) + slack
    for fr in hello:
        content = fr[8:]
        assert len(content) == 44
        lib.val_deserialize_handshake(content, hs)
        magic, vmaj, vmin, _, packet_size = struct.unpack_from("<IBBHI", hs.raw)
        assert magic == 0x56414C00 and (vmaj, vmin) == (0, 7) and packet_size == 1024
        out = ctypes.create_string_buffer(44)
        lib.val_serialize_handshake(hs, out)
        assert out.raw == content
    meta = _ctrl_frames(2)
    assert meta
    for fr in meta:
        content = fr[8:]
        assert len(content) == 264
        m = ctypes.create_string_buffer(272)
        lib.val_deserialize_meta(content, m)
        assert m.raw[:9] == b"input.bin"
        out = ctypes.create_string_buffer(264)
        lib.val_serialize_meta(m, out)
        assert out.raw == content
    for fr in _ctrl_frames(4):  # RESUME_RESP, if the transfer had one
        content = fr[8:]
        r = ctypes.create_string_buffer(40)
        lib.val_deserialize_resume_resp(content, r)
        out = ctypes.create_string_buffer(24)
        lib.val_serialize_resume_resp(r, out)
        assert out.raw == content[:24]


# ---- against the reference tree (build container only) ----------------------
def _public_macros():
    names = []
    for h in ("val_protocol.h", "val_wire.h", "val_errors.h"):
        for m in re.finditer(r"^\s*#\s*define\s+(VAL_[A-Z0-9_]+)\s+\S", open(os.path.join(REF, "include", h)).read(),
                             re.M):
            names.append(m.group(1))
    return sorted(set(names) - {"VAL_PROTOCOL_H", "VAL_WIRE_H", "VAL_ERRORS_H"})


_LAYOUT = {
    "val_config_t": ["transport", "filesystem", "crc32_provider", "system", "timeouts", "features", "retries",
                     "buffers", "resume", "tx_flow", "callbacks", "metadata_validation", "debug", "capture"],
    "val_handshake_t": ["magic", "version_major", "version_minor", "reserved", "packet_size", "features", "required",
                        "requested", "tx_max_window_packets", "rx_max_window_packets", "ack_stride_packets",
                        "reserved_capabilities", "supported_features16", "required_features16",
                        "requested_features16", "reserved2"],
    "val_error_payload_t": ["code", "detail"],
    "val_resume_resp_t": ["action", "resume_offset", "verify_crc", "verify_length"],
    "val_meta_payload_t": ["filename", "sender_path", "file_size"],
    "val_packet_record_t": ["direction", "type", "wire_len", "payload_len", "offset", "crc_ok", "timestamp_ms",
                            "session_id"],
    "val_resume_config_t": ["mode", "tail_cap_bytes", "min_verify_bytes", "mismatch_skip"],
    "val_tx_flow_config_t": ["window_cap_packets", "initial_cwnd_packets", "retransmit_cache_enabled",
                             "degrade_error_threshold", "recovery_success_threshold", "allocator"],
    "val_progress_info_t": ["bytes_transferred", "total_bytes", "current_file_bytes", "files_completed",
                            "total_files", "transfer_rate_bps", "eta_seconds", "current_filename"],
    "val_error_t": ["code", "detail", "op"],
    "val_metrics_t": ["packets_sent", "send_by_type", "recv_by_type", "timeouts", "crc_errors", "rtt_samples"],
}
_ENUMS = ["VAL_PKT_HELLO", "VAL_PKT_DATA", "VAL_PKT_DATA_NAK", "VAL_ACK_FLAG_EOF", "VAL_RESUME_TAIL",
          "VAL_RESUME_VERIFY_FIRST", "VAL_RESUME_ABORT_FILE", "VAL_LOG_TRACE", "VAL_DIR_RX", "VAL_VALIDATION_ABORT",
          "VAL_ERR_PERFORMANCE", "VAL_ERR_UNSUPPORTED_TX_MODE", "VAL_SKIPPED"]


def _dumper_source():
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "val_protocol.h"', '#include "val_wire.h"',
             "int main(void) {"]
    for t, fields in _LAYOUT.items():
        lines.append(f'printf("sizeof {t} %zu\\n", sizeof({t}));')
        for f in fields:
            lines.append(f'printf("offsetof {t}.{f} %zu\\n", offsetof({t}, {f}));')
    for e in _ENUMS:
        lines.append(f'printf("enum {e} %lld\\n", (long long)({e}));')
    for m in _public_macros():
        lines.append(f'printf("macro {m} %llu\\n", (unsigned long long)({m}));')
    lines += ["return 0;", "}"]
    return "\n".join(lines)


@needs_gcc
@needs_ref
def test_layouts_enums_and_macros_equal_reference():
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "dump.c"), "w").write(_dumper_source())
        out = {}
        for tag, inc in (("ref", os.path.join(REF, "include")), ("ours", INC)):
            _gcc(["-std=gnu99", "-DVAL_ENABLE_METRICS=1", f"-I{inc}", "dump.c", "-o", tag], cwd=d)
            out[tag] = _run(os.path.join(d, tag)).splitlines()
    assert len(out["ref"]) > 150
    diff = [(a, b) for a, b in zip(out["ref"], out["ours"]) if a != b]
    assert not diff and len(out["ref"]) == len(out["ours"]), diff[:10]


@needs_gcc
@needs_ref
def test_reference_sources_compile_against_our_headers():
    with tempfile.TemporaryDirectory() as d:
        for src in REF_SRCS:
            _gcc(["-std=gnu99", "-O1", "-DVAL_ENABLE_METRICS=1", "-DVAL_LOG_LEVEL=0",
                  "-Werror=implicit-function-declaration", "-Werror=incompatible-pointer-types",
                  "-Werror=int-conversion", f"-I{INC}", f"-I{REF}/src", "-c", src, "-o",
                  os.path.join(d, os.path.basename(src) + ".o")])


@needs_gcc
@needs_ref
def test_reference_protocol_over_our_headers_regenerates_fixtures():
    """The reference's sender/receiver/core, built against include/, produce
    the same golden frames, verdicts, loopback log and ABI block as when built
    against the reference's own headers."""
    with tempfile.TemporaryDirectory() as d:
        flags = ["-std=gnu99", "-O2", "-w", "-DVAL_ENABLE_METRICS=1", "-DVAL_LOG_LEVEL=0", f"-I{INC}",
                 f"-I{REF}/src", f"-I{ROOT}/oracle"]
        _gcc([*flags, "-o", os.path.join(d, "gen"), os.path.join(ROOT, "oracle", "gen_golden.c"), *REF_SRCS,
              "-lpthread"])
        _gcc([*flags, "-o", os.path.join(d, "harness"), os.path.join(ROOT, "oracle", "provider_harness.c"), *REF_SRCS,
              "-ldl", "-lpthread"])
        ref_vectors = _run(os.path.join(d, "gen"))
        dropin = _run(os.path.join(d, "harness"), "none", "fixtures")
    assert ref_vectors == open(os.path.join(ROOT, "tests", "golden", "ref_vectors.json")).read()
    assert dropin == open(os.path.join(ROOT, "tests", "golden", "dropin_vectors.json")).read()


_CODEC_DRIVER = r"""
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "val_wire.h"
static unsigned long long s = 0x9E3779B97F4A7C15ull;
static unsigned long long rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static void fill(void *p, size_t n) { unsigned char *c = p; for (size_t i = 0; i < n; i++) c[i] = (unsigned char)rnd(); }
static void hex(const unsigned char *b, size_t n) { for (size_t i = 0; i < n; i++) printf("%02x", b[i]); printf("\n"); }
int main(void) {
    unsigned char w[512];
    for (int it = 0; it < 200; it++) {
        val_handshake_t hs; fill(&hs, sizeof hs);
        memset(w, 0xAA, sizeof w); val_serialize_handshake(&hs, w); hex(w, VAL_WIRE_HANDSHAKE_SIZE);
        val_handshake_t h2; memset(&h2, 0, sizeof h2); val_deserialize_handshake(w, &h2);
        memset(w, 0xAA, sizeof w); val_serialize_handshake(&h2, w); hex(w, VAL_WIRE_HANDSHAKE_SIZE);
        val_meta_payload_t m; fill(&m, sizeof m);
        memset(w, 0xAA, sizeof w); val_serialize_meta(&m, w); hex(w, VAL_WIRE_META_SIZE);
        val_meta_payload_t m2; memset(&m2, 0, sizeof m2); val_deserialize_meta(w, &m2);
        printf("%d\n", memcmp(&m, &m2, offsetof(val_meta_payload_t, file_size)) == 0 && m.file_size == m2.file_size);
        val_resume_resp_t r; memset(&r, 0, sizeof r); r.action = (val_resume_action_t)(rnd() % 5);
        r.resume_offset = rnd(); r.verify_crc = (unsigned)rnd(); r.verify_length = rnd();
        memset(w, 0xAA, sizeof w); val_serialize_resume_resp(&r, w); hex(w, VAL_WIRE_RESUME_RESP_SIZE);
        val_resume_resp_t r2; val_deserialize_resume_resp(w, &r2);
        printf("%d %llu %u %llu\n", (int)r2.action, (unsigned long long)r2.resume_offset, r2.verify_crc,
               (unsigned long long)r2.verify_length);
        unsigned long long off = rnd(); unsigned crc = (unsigned)rnd(), len = (unsigned)rnd();
        memset(w, 0xAA, sizeof w); val_serialize_verify_request(off, crc, len, w); hex(w, VAL_WIRE_VERIFY_REQ_SIZE);
        unsigned long long o2 = 0; unsigned c2 = 0, l2 = 0; val_deserialize_verify_request(w, &o2, &c2, &l2);
        printf("%llu %u %u\n", o2, c2, l2);
        val_status_t st = (val_status_t)(-(int)(rnd() % 16));
        memset(w, 0xAA, sizeof w); val_serialize_verify_response(st, crc, w); hex(w, VAL_WIRE_VERIFY_RESP_SIZE);
        val_status_t st2; unsigned rc2; val_deserialize_verify_response(w, &st2, &rc2); printf("%d %u\n", (int)st2, rc2);
        val_error_payload_t e; e.code = (int)rnd(); e.detail = (unsigned)rnd();
        memset(w, 0xAA, sizeof w); val_serialize_error_payload(&e, w); hex(w, VAL_WIRE_ERROR_PAYLOAD_SIZE);
        val_error_payload_t e2; val_deserialize_error_payload(w, &e2); printf("%d %u\n", e2.code, e2.detail);
        unsigned char hdr[8]; val_serialize_frame_header((unsigned char)rnd(), (unsigned char)rnd(),
                                                         (unsigned short)rnd(), (unsigned)rnd(), hdr);
        hex(hdr, 8);
    }
    val_serialize_handshake(NULL, w); val_deserialize_handshake(NULL, NULL); val_serialize_meta(NULL, w);
    val_deserialize_verify_request(NULL, NULL, NULL, NULL); val_serialize_error_payload(NULL, NULL);
    printf("null-ok\n");
    return 0;
}
"""


@needs_gcc
@needs_ref
def test_codec_bytes_equal_reference_codec():
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "drv.c"), "w").write(_CODEC_DRIVER)
        common = ["-std=gnu99", "-O2", "-Wall", "-Wno-unused-function", f"-I{INC}", "drv.c"]
        _gcc([*common, os.path.join(REF, "src", "val_wire.c"), "-o", "ref"], cwd=d)
        _gcc([*common, os.path.join(ROOT, "val_protocol_amd", "csrc", "val_wire.c"), "-o", "ours"], cwd=d)
        a, b = _run(os.path.join(d, "ref")), _run(os.path.join(d, "ours"))
    assert a.count("\n") > 2000 and a.endswith("null-ok\n")
    assert a == b
