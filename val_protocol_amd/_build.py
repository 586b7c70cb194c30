"""Build recipe for libval_crc_hip.so (gfx950). Invoked by __graft_entry__.build()
and, on demand, by ``crc.lib()`` when the library is missing or was built from
other sources (a content stamp, not mtimes: a gpurun snapshot does not keep
them)."""
from __future__ import annotations

import fcntl
import glob
import hashlib
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "val_protocol_amd", "csrc")
INC = os.path.join(ROOT, "include")
BUILD = os.path.join(ROOT, "build")
OUT = os.path.join(ROOT, "val_protocol_amd", "libval_crc_hip.so")
ARCH = "gfx950"


def _run(cmd, verbose):
    if verbose:
        print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def sources() -> list[str]:
    """Every file the library is built from (sources, headers, this recipe)."""
    files = sorted(glob.glob(os.path.join(CSRC, "*"))) + sorted(glob.glob(os.path.join(INC, "*.h")))
    return [f for f in files if os.path.isfile(f)] + [os.path.abspath(__file__)]


def source_hash() -> str:
    h = hashlib.sha256()
    for f in sources():
        h.update(os.path.relpath(f, ROOT).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def stamp_path(out: str) -> str:
    return out + ".srchash"


def is_current(out: str = OUT) -> bool:
    """The library exists and was built from the sources in this tree."""
    try:
        with open(stamp_path(out)) as fh:
            return os.path.exists(out) and fh.read().strip() == source_hash()
    except OSError:
        return False


def build(verbose: bool = True, out: str = OUT, build_dir: str = BUILD) -> str:
    """Compile val_wire.c, val_batch.c and cpu_crc32.c (gcc) and val_crc32_hip.hip (hipcc, gfx950) and link
    ``out``. The library is linked to a temporary name and renamed, so a
    process that loads ``out`` meanwhile never sees a half-written file."""
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    os.makedirs(build_dir, exist_ok=True)
    digest = source_hash()
    wire_o = os.path.join(build_dir, "val_wire.o")
    hip_o = os.path.join(build_dir, "val_crc32_hip.o")
    cpu_o = os.path.join(build_dir, "cpu_crc32.o")
    batch_o = os.path.join(build_dir, "val_batch.o")
    _run(["gcc", "-O2", "-fPIC", "-std=c99", "-Wall", "-Wextra", "-Werror", f"-I{INC}", "-c",
          os.path.join(CSRC, "val_wire.c"), "-o", wire_o], verbose)
    _run(["gcc", "-O3", "-fPIC", "-std=gnu99", "-Wall", "-Wextra", "-Werror", f"-I{CSRC}", "-c",
          os.path.join(CSRC, "cpu_crc32.c"), "-o", cpu_o], verbose)
    _run(["gcc", "-O2", "-fPIC", "-std=c99", "-Wall", "-Wextra", "-Werror", f"-I{INC}", "-c",
          os.path.join(CSRC, "val_batch.c"), "-o", batch_o], verbose)
    hip_cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", "-Werror", f"-I{INC}",
               f"-I{CSRC}", "-c", os.path.join(CSRC, "val_crc32_hip.hip"), "-o", hip_o]
    # The HIP object takes minutes: it is rebuilt only when a file it includes
    # (every header and the .hip itself) or its command changed.
    hip_stamp = hip_o + ".srchash"
    h = hashlib.sha256(" ".join(hip_cmd).encode())
    for f in sources():
        if not f.endswith(".c") and not f.endswith(".py"):
            h.update(os.path.relpath(f, ROOT).encode())
            with open(f, "rb") as fh:
                h.update(fh.read())
    hip_digest = h.hexdigest()
    try:
        with open(hip_stamp) as fh:
            hip_current = os.path.exists(hip_o) and fh.read().strip() == hip_digest
    except OSError:
        hip_current = False
    if not hip_current:
        _run(hip_cmd, verbose)
        with open(hip_stamp, "w") as fh:
            fh.write(hip_digest + "\n")
    fd, tmp = tempfile.mkstemp(prefix=".libval_crc_hip.", suffix=".so", dir=os.path.dirname(out))
    os.close(fd)
    try:
        _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-Wl,--no-undefined", "-o", tmp, hip_o, wire_o, cpu_o, batch_o,
              "-lpthread"], verbose)
        os.chmod(tmp, 0o755)
        os.replace(tmp, out)
    finally:
        if os.path.exists(tmp):
            os.unlink(tmp)
    with open(stamp_path(out), "w") as fh:
        fh.write(digest + "\n")
    return out


def ensure_built(verbose: bool = False) -> str:
    """Build OUT under a file lock unless it is current (concurrent test
    processes build once)."""
    if is_current():
        return OUT
    lock = os.path.join(os.path.dirname(OUT), ".build.lock")
    with open(lock, "w") as fh:
        fcntl.flock(fh, fcntl.LOCK_EX)
        try:
            if not is_current():
                build(verbose=verbose)
        finally:
            fcntl.flock(fh, fcntl.LOCK_UN)
    return OUT


if __name__ == "__main__":
    build(verbose="-q" not in sys.argv)
