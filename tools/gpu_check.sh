# Health check of the tree on one MI355X: GPU parity tests, smoke, headline bench
# (+ cfg5, cfg2). Test failures (pytest rc 1) still run the bench; any other
# failure (timeout, abort, fault) ends the script there.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/check
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 600 python bench.py --config cfg5 --no-cpu-baseline > $O/bench_cfg5.json 2> $O/bench_cfg5.err && \
timeout -k 10 600 python bench.py --config cfg2 --no-cpu-baseline --steps 200 > $O/bench_cfg2.json 2> $O/bench_cfg2.err
rc2=$?; echo "check rc=$rc2"; cat $O/bench*.json; exit $rc2
