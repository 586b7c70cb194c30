set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2_pytest.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r2_bench.log 2>&1
rc=$?; tail -5 gpurun_out/r2_pytest.log; tail -3 gpurun_out/r2_smoke.log; tail -3 gpurun_out/r2_bench.log; exit $rc
