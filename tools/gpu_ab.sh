# Same-box A/B on the GPU box (tooling only): build/libval_A.so against each
# build/libval_<V>.so named in $LIBS (default "B"; tools/build_rev.sh builds
# them from any revision or -D variant) on the workloads given as arguments
# (tools/ab_libs.py names). Optional steps, each under its own time limit and
# chained so a failure ends the call:
#   TESTS=1   the GPU test suite first (the in-tree library)
#   REGION=1  region-window A/B (tools/ab_region.py)
#   HDR=1     cfg3b with header_crc as well
#   MICRO="mb13 mb14"  micro-benchmarks from bench/micro first
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab
mkdir -p $O
rc=0
for m in ${MICRO:-}; do
  timeout -k 10 200 $R/bench/micro/$m > $O/$m.log 2>&1 || { rc=$?; echo "$m failed"; exit $rc; }
  grep -v amdgpu.ids $O/$m.log
done
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
libs=""; for v in ${LIBS:-B}; do libs="$libs build/libval_$v.so"; done
if [ "${REGION:-0}" = 1 ]; then
  timeout -k 10 300 python tools/ab_region.py build/libval_A.so $libs > $O/ab_region.log 2>&1 || exit 1
  grep -v amdgpu.ids $O/ab_region.log
fi
if [ $# -gt 0 ]; then
  timeout -k 10 900 python tools/ab_libs.py build/libval_A.so $libs "$@" > $O/ab.log 2>&1 || exit 1
  grep -v amdgpu.ids $O/ab.log | cut -c1-220
fi
if [ "${HDR:-0}" = 1 ]; then
  AB_HDR=1 timeout -k 10 300 python tools/ab_libs.py build/libval_A.so $libs cfg3b > $O/ab_hdr.log 2>&1 || exit 1
  grep -v amdgpu.ids $O/ab_hdr.log | cut -c1-220
fi
echo "rc=0"
