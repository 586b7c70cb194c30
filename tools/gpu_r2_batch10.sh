set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_pytest.log 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py build/ab/head.so build/ab/new.so cfg2 w256 cfg3b > gpurun_out/ab_frames.log 2>&1 && \
timeout -k 10 300 python tools/ab_region.py build/ab/head.so build/ab/new.so > gpurun_out/ab_region5.log 2>&1 && \
timeout -k 10 300 python tools/region_latency.py > gpurun_out/r2_region.log 2>&1
rc=$?
tail -2 gpurun_out/r2_pytest.log; cat gpurun_out/ab_frames.log gpurun_out/ab_region5.log gpurun_out/r2_region.log
exit $rc
