"""The drop-in boundary: the C-ABI library loads, exports every function the
public headers declare, and the public struct layout equals the reference's
(golden abi block, measured on the reference headers)."""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

import val_protocol_amd.crc as vc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")


def _declared_functions():
    names = set()
    for h in ("val_crc32_gpu.h", "val_protocol.h", "val_wire.h", "val_batch.h"):
        txt = open(os.path.join(INC, h)).read()
        # the session API is the reference's control plane, declared for its sources, not exported here
        txt = re.sub(r"/\* control-plane API begin \*/.*?/\* control-plane API end \*/", "", txt, flags=re.S)
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        txt = re.sub(r"static inline[^{]*\{[^}]*\}", "", txt)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_]*\s*\**\s*\b(val_[a-z0-9_]+)\s*\(", txt, re.M):
            if not m.group(0).lstrip().startswith("typedef") and not m.group(1).endswith("_t"):
                names.add(m.group(1))
    return names


def test_library_loads_and_exports_everything():
    lib = vc.lib()
    declared = _declared_functions()
    assert declared, "header parse found nothing"
    missing = [n for n in sorted(declared) if not hasattr(lib, n)]
    assert not missing, f"declared but not exported: {missing}"
    assert set(vc.EXPORTS) >= declared
    assert lib.val_gpu_abi_version() == 1


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_struct_layout_matches_reference(golden):
    src = r"""
    #include "val_protocol.h"
    #include "val_wire.h"
    #include "val_crc32_gpu.h"
    #include <stdio.h>
    int main(void) {
        val_config_t cfg = {0};
        cfg.crc32_provider = val_gpu_crc32_provider;  /* the drop-in */
        (void)cfg;
        printf("%zu %zu %zu %zu\n", sizeof(val_config_t), offsetof(val_config_t, crc32_provider),
               sizeof(val_packet_record_t), offsetof(val_config_t, buffers));
        return 0;
    }
    """
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        libdir = os.path.dirname(vc.LIB_PATH)
        subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", f"-I{INC}", c, "-o", exe, f"-L{libdir}",
                        "-l:libval_crc_hip.so", f"-Wl,-rpath,{libdir}", "-Wl,--unresolved-symbols=ignore-in-shared-libs"],
                       check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    abi = golden["abi"]
    assert [int(x) for x in out] == [abi["sizeof_val_config_t"], abi["offsetof_crc32_provider"],
                                     abi["sizeof_val_packet_record_t"], abi["offsetof_buffers"]]


def test_no_gpu_means_loud_failure_not_fallback():
    if vc.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(vc.ValError) as e:
        vc.init(0)
    assert e.value.status == vc.VAL_ERR_IO


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_batch_attach_argument_checks():
    """val_batch_attach (include/val_batch.h) refuses configs the provider
    could not tell apart: one buffer for both directions, or a buffer that
    another attached config already uses, and a tx/rx that is not a
    VAL_BATCH_* mode; detach restores the hooks. No
    GPU needed (the window buffers are plain host memory then)."""
    src = r"""
    #include "val_batch.h"
    #include <stdio.h>
    #include <string.h>
    static int snd(void *c, const void *d, size_t n) { (void)c; (void)d; return (int)n; }
    static int rcv(void *c, void *b, size_t n, size_t *g, unsigned t) { (void)c; (void)b; (void)n; (void)t; *g = 0; return 0; }
    static char a[2048], b[2048], c[2048];
    int main(void) {
        val_config_t x, y;
        memset(&x, 0, sizeof x);
        x.transport.send = snd;
        x.transport.recv = (int (*)(void *, void *, size_t, size_t *, uint32_t))rcv;
        x.buffers.packet_size = 2048;
        x.buffers.send_buffer = a;
        x.buffers.recv_buffer = a;
        val_batch_t *bx = NULL, *by = NULL;
        int r1 = val_batch_attach(&x, NULL, &bx);          /* same buffer both ways */
        x.buffers.recv_buffer = b;
        int r2 = val_batch_attach(&x, NULL, &bx);          /* fine */
        int hooked = x.transport.send != snd && x.crc32_provider == val_batch_crc32_provider;
        y = x;
        y.transport.send = snd;
        y.buffers.send_buffer = c;                          /* recv_buffer b is taken */
        int r3 = val_batch_attach(&y, NULL, &by);
        val_batch_detach(bx);
        int restored = x.transport.send == snd && x.crc32_provider == NULL;
        int r4 = val_batch_attach(&y, NULL, &by);          /* b is free again */
        val_batch_detach(by);
        val_batch_opts_t o;
        memset(&o, 0, sizeof o);
        o.tx = VAL_BATCH_ALWAYS + 1;                        /* not a mode */
        y.transport.send = snd;
        int r5 = val_batch_attach(&y, &o, &by);
        o.tx = VAL_BATCH_ALWAYS;
        o.rx = VAL_BATCH_OFF;
        int r6 = val_batch_attach(&y, &o, &by);
        val_batch_detach(by);
        printf("%d %d %d %d %d %d %d %d %d\n", r1, r2, hooked, r3, restored, r4, r5, r6,
               VAL_BATCH_OFF * 100 + VAL_BATCH_AUTO * 10 + VAL_BATCH_ALWAYS);
        return 0;
    }
    """
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        libdir = os.path.dirname(vc.LIB_PATH)
        vc.lib()  # built and current
        subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", f"-I{INC}", c, "-o", exe, f"-L{libdir}",
                        "-l:libval_crc_hip.so", f"-Wl,-rpath,{libdir}"], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    assert [int(v) for v in out] == [vc.VAL_ERR_INVALID_ARG, 0, 1, vc.VAL_ERR_INVALID_ARG, 1, 0,
                                     vc.VAL_ERR_INVALID_ARG, 0, 12]


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_batch_registry_capacity_and_reuse():
    """Up to 256 attached configs per process (include/val_batch.h): the 257th
    attach is refused, detaching frees the slots for reuse, and the provider
    on a buffer of no attached config answers with the plain CRC."""
    src = r"""
    #include "val_batch.h"
    #include <stdio.h>
    #include <string.h>
    #include <stdlib.h>
    static int snd(void *c, const void *d, size_t n) { (void)c; (void)d; return (int)n; }
    static int rcv(void *c, void *b, size_t n, size_t *g, uint32_t t) { (void)c; (void)b; (void)n; (void)t; *g = 0; return 0; }
    int main(void) {
        static val_config_t cfg[257];
        static char buf[257][2][64];
        val_batch_t *b[257];
        val_batch_opts_t o;
        memset(&o, 0, sizeof o);
        o.max_frames = 4;
        o.max_bytes = 64;
        int ok = 0;
        for (int i = 0; i < 257; i++) {
            memset(&cfg[i], 0, sizeof cfg[i]);
            cfg[i].transport.send = snd;
            cfg[i].transport.recv = rcv;
            cfg[i].buffers.packet_size = 64;
            cfg[i].buffers.send_buffer = buf[i][0];
            cfg[i].buffers.recv_buffer = buf[i][1];
            b[i] = NULL;
            ok += val_batch_attach(&cfg[i], &o, &b[i]) == 0;
        }
        const char kat[] = "123456789";
        unsigned plain = val_batch_crc32_provider(0xFFFFFFFFu, kat, 9);
        for (int i = 0; i < 256; i++) val_batch_detach(b[i]);
        int again = val_batch_attach(&cfg[256], &o, &b[256]) == 0;
        val_batch_detach(b[256]);
        printf("%d %d %08x\n", ok, again, plain);
        return 0;
    }
    """
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(src)
        exe = os.path.join(d, "t")
        libdir = os.path.dirname(vc.LIB_PATH)
        vc.lib()
        subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", f"-I{INC}", c, "-o", exe, f"-L{libdir}",
                        "-l:libval_crc_hip.so", f"-Wl,-rpath,{libdir}"], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout.split()
    assert out == ["256", "1", "cbf43926"]
