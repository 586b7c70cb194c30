# GPU tests, region A/B (build/libval_A.so vs build/libval_B.so) and a frames A/B. Tooling only.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/fc; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python tools/ab_region.py build/libval_A.so build/libval_B.so > $O/ab_region.log 2>&1 && \
timeout -k 10 600 python tools/ab_libs.py build/libval_A.so build/libval_B.so w256x16400 w64x65536 cfg2 cfg5log s1100 > $O/ab.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; grep -v amdgpu $O/ab_region.log $O/ab.log; echo rc=$rc; exit $rc
