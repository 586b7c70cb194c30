# GPU tests, then a same-box A/B (build/libval_A.so vs build/libval_B.so) on
# the workloads given, plus cfg3b with header_crc. Tooling only.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python tools/ab_libs.py build/libval_A.so build/libval_B.so "$@" > $O/ab.log 2>&1 && \
AB_HDR=1 timeout -k 10 300 python tools/ab_libs.py build/libval_A.so build/libval_B.so cfg3b > $O/ab_hdr.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; grep -v amdgpu.ids $O/ab.log $O/ab_hdr.log; echo "rc=$rc"; exit $rc
