set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_pytest.log 2>&1 && \
timeout -k 10 300 python tools/ab_region.py build/ab/base.so build/ab/new.so > gpurun_out/ab_region3.log 2>&1 && \
timeout -k 10 120 python tools/timing_region.py build/ab/timing.so 262144 1048576 8388608 67108864 > gpurun_out/r2_timing_region.log 2>&1 && \
timeout -k 10 300 python tools/region_latency.py > gpurun_out/r2_region.log 2>&1
rc=$?
tail -3 gpurun_out/r2_pytest.log; cat gpurun_out/ab_region3.log gpurun_out/r2_timing_region.log gpurun_out/r2_region.log
exit $rc
