# Round 6: in-launch tail pieces of 1 KiB. Tail and parity tests, then the
# same-box A/B: A = the previous library (a second launch for the tail), B =
# 4 KiB pieces, C = this tree (1 KiB pieces, doubled when needed).
set -o pipefail
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_tail.py \
    tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_split.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python tools/ab_libs.py build/libA_r6.so build/libB_r6.so build/libC_r6.so cfg3b cfg4d t16390 t32779 t65557 cfg3b t16390 > $O/ab.log 2>&1 || exit 4
cat $O/ab.log
