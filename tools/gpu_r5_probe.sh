# Round-5 probe: k_region_dyn parity (region tests) and its same-box A/B
# against the one-chunk-per-wave k_region (build/libval_A.so).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/g7; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k region -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -4 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab_region.py build/libval_A.so build/libval_B.so 8388608 33554432 67108864 134217728 268435456 1073741824 > $O/ab_region.log 2>&1
rc=$?; grep -v amdgpu $O/ab_region.log; exit $rc
