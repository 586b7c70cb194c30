# Same-box A/B/C of build/libval_{A,B,C}.so on the workloads given (no test run). Tooling only.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab; mkdir -p $O
timeout -k 10 600 python tools/ab_libs.py build/libval_A.so build/libval_B.so build/libval_C.so "$@" > $O/ab3.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab3.log; echo "rc=$rc"; exit $rc
