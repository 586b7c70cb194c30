#!/bin/bash
# One rocprofv3 kernel-trace run per workload spec (tools/prof_small.py), so
# kernels of different workloads are not merged. usage: OUTDIR LIB spec...
set -uo pipefail
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/$1; LIB=$2; shift 2
mkdir -p "$OUT"
for spec in "$@"; do
  d="$OUT/${spec//:/_}"
  VCRC_LIB=$R/$LIB timeout -k 10 120 rocprofv3 --kernel-trace -d "$d" -o run -- python3 "$R/tools/prof_small.py" 20 "$spec" > "$d.log" 2>&1 || exit 1
  echo "== $spec"; python3 "$R/tools/rocpd_kernels.py" "$(find "$d" -name '*.db' | head -1)" | grep -v "at::native\|rocclr"
done
