set -o pipefail
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/slice_probe.py > $O/slice_probe.jsonl 2> $O/slice_probe.err || exit 4
cat $O/slice_probe.jsonl
