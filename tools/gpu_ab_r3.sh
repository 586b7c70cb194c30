# GPU tests, then a same-box A/B (build/libval_A.so vs build/libval_B.so) on
# the workloads given, then the traffic of u1100d with the product library.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 600 python tools/ab_libs.py build/libval_A.so build/libval_B.so "$@" > $O/ab.log 2>&1 && \
bash tools/pmc_variants.sh u1100d "VAL_GPU_X=0" "VAL_GPU_CARRY=0" > $O/pmcv.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; grep -v amdgpu.ids $O/ab.log; echo "rc=$rc"; exit $rc
