#!/bin/bash
# rocprofv3 kernel durations of small-batch workloads for several library
# builds (tools/prof_small.py), plus an optional micro-benchmark binary.
# usage: tools/gpu_prof_ab.sh OUTDIR "workload specs" lib1.so [lib2.so ...] [-- ./bench/micro/mbN]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/$1; SPECS=$2; shift 2
mkdir -p "$OUT"
i=0
while [ $# -gt 0 ] && [ "$1" != "--" ]; do
  lib=$1; shift; i=$((i+1))
  VCRC_LIB=$R/$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/l$i" -o run -- python3 "$R/tools/prof_small.py" 30 $SPECS > "$OUT/l$i.log" 2>&1
  echo "== $lib"; python3 "$R/tools/rocpd_kernels.py" "$(find "$OUT/l$i" -name '*.db' | head -1)"
done
if [ "${1:-}" = "--" ]; then shift
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/micro" -o run -- "$R/$1" > "$OUT/micro.log" 2>&1
  echo "== $1"; python3 "$R/tools/rocpd_kernels.py" "$(find "$OUT/micro" -name '*.db' | head -1)"
fi
