#!/bin/bash
# Build libval_crc_hip.so from the csrc/ of git revision $1 (or "WT" = working
# tree) into $2, for same-box A/B runs with tools/ab_libs.py. Tooling only.
set -euo pipefail
REV=$1; OUT=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
if [ "$REV" = "WT" ]; then cp -r "$ROOT/val_protocol_amd/csrc" "$T/csrc"; cp -r "$ROOT/include" "$T/include"
else mkdir -p "$T/csrc" "$T/include"
  git -C "$ROOT" archive "$REV" val_protocol_amd/csrc include | tar -x -C "$T"
  mv "$T/val_protocol_amd/csrc/"* "$T/csrc/"; fi
gcc -O2 -fPIC -std=c99 -I"$T/include" -c "$T/csrc/val_wire.c" -o "$T/w.o"
X=""; if [ -f "$T/csrc/cpu_crc32.c" ]; then gcc -O3 -fPIC -std=gnu99 -I"$T/csrc" -c "$T/csrc/cpu_crc32.c" -o "$T/c.o"; X="$T/c.o"; fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -I"$T/include" -I"$T/csrc" -c "$T/csrc/val_crc32_hip.hip" -o "$T/h.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" "$T/h.o" "$T/w.o" $X -lpthread
rm -rf "$T"; echo "built $REV -> $OUT"
