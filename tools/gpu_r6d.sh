# Round 6: in-launch tail pieces. GPU suite (with tests/test_gpu_tail.py),
# same-box A/B of the previous library (A) against this tree (B) on cfg3, the
# cfg4 file and its slices, then a driver-style bench line.
set -o pipefail
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python tools/ab_libs.py build/libA_r6.so build/libB_r6.so cfg3b cfg4d t16390 t32779 t65557 cfg3b > $O/ab.log 2>&1 || exit 4
cat $O/ab.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 5
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; s=d['cfg4_strong']; print(d['value'], r['kernel_ms'], r['frac'], r['read_roof'], '| block', s['per_rank'][0]['kernel_ms'], s['roofline']['frac'], '| proxy', {k:(v['kernel_ms'], v['est_aggregate_GiB_s']) for k,v in d['cfg4_strong_proxy'].items() if k in '1248'})"
