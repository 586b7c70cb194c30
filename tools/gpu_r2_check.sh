# Round-2 GPU check: full GPU suite, smoke, headline bench, and the RX verify
# lines (with and without the payload-state by-product). Writes gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2_pytest.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2_smoke.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/r2_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --verify --no-cpu-baseline >> gpurun_out/r2_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --verify --pay --no-cpu-baseline >> gpurun_out/r2_bench.log 2>&1
rc=$?
tail -3 gpurun_out/r2_pytest.log; tail -1 gpurun_out/r2_smoke.log
grep -o '"workload": "[^"]*"\|"kernel_ms": [0-9.]*' gpurun_out/r2_bench.log
exit $rc
