# Quick health check of the tree on one MI355X: GPU parity tests, smoke, headline bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/check
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 600 python bench.py --config cfg5 --no-cpu-baseline > $O/bench_cfg5.json 2> $O/bench_cfg5.err && \
timeout -k 10 600 python bench.py --config cfg2 --no-cpu-baseline --steps 200 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
rc=$?; echo "check rc=$rc"; tail -3 $O/pytest_gpu.log; cat $O/bench*.json; exit $rc
