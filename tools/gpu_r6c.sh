# Round 6: the batcher's session tests and the proxy test on the GPU, a
# driver-style bench line, and a kernel trace of the cfg4 slice probe.
set -o pipefail
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests/test_dropin_sessions.py \
    tests/test_gpu_multiproc.py > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 5
python3 -c "import json; d=json.load(open('$O/bench.json')); r=d['roofline']; s=d['cfg4_strong']; print(d['value'], r['kernel_ms'], r['frac'], r['read_roof'], '| block', s['per_rank'][0]['kernel_ms'], s['roofline']['frac'], s['warmup_launches'], '| proxy', {k:(v['kernel_ms'], v['est_aggregate_GiB_s']) for k,v in d['cfg4_strong_proxy'].items() if k in '1248'})"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o slice -- python3 $GRAFT_REPO_ROOT/tools/slice_probe.py --steps 10 > $GRAFT_REPO_ROOT/$O/trace.log 2>&1
echo "trace rc=$?"
