set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2_pytest.log 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py build/ab/head.so build/ab/new.so cfg2 w256 cfg3b cfg4 cfg5log > gpurun_out/ab_prologue.log 2>&1 && \
timeout -k 10 300 python tools/ab_region.py build/ab/head.so build/ab/new.so > gpurun_out/ab_region4.log 2>&1 && \
timeout -k 10 120 python tools/timing_cfg2.py build/ab/timing.so cfg2 4 > gpurun_out/r2_timing_cfg2.log 2>&1 && \
timeout -k 10 120 python tools/timing_region.py build/ab/timing.so 1048576 8388608 > gpurun_out/r2_timing_region.log 2>&1
rc=$?
tail -2 gpurun_out/r2_pytest.log; cat gpurun_out/ab_prologue.log gpurun_out/ab_region4.log gpurun_out/r2_timing_cfg2.log gpurun_out/r2_timing_region.log
exit $rc
