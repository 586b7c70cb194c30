"""Build recipe for libval_crc_hip.so (gfx950). Invoked by __graft_entry__.build()."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

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


def build(verbose: bool = True) -> str:
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    os.makedirs(BUILD, exist_ok=True)
    wire_o = os.path.join(BUILD, "val_wire.o")
    hip_o = os.path.join(BUILD, "val_crc32_hip.o")
    _run(["gcc", "-O2", "-fPIC", "-std=c99", "-Wall", "-Wextra", "-Werror", f"-I{INC}", "-c",
          os.path.join(CSRC, "val_wire.c"), "-o", wire_o], verbose)
    _run([hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall", f"-I{INC}", f"-I{CSRC}", "-c",
          os.path.join(CSRC, "val_crc32_hip.hip"), "-o", hip_o], verbose)
    _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT, hip_o, wire_o], verbose)
    return OUT


if __name__ == "__main__":
    build(verbose="-q" not in sys.argv)
