# Round 3: mb13 short-frame read patterns (MB13=0 skips them), GPU parity of the working tree, and
# a same-box A/B of build/libval_{A,B}.so on short and long batches. Tooling only.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r3q; mkdir -p $O
if [ "${MB13:-1}" = 1 ]; then
  timeout -k 10 120 $R/bench/micro/mb13 > $O/mb13.log 2>&1 || { echo "mb13 failed"; exit 1; }
  grep -v amdgpu.ids $O/mb13.log
fi
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_round3.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_fuzz.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/ab_libs.py build/libval_A.so build/libval_B.so "$@" > $O/ab.log 2>&1
rc=$?; grep -v amdgpu.ids $O/ab.log; exit $rc
