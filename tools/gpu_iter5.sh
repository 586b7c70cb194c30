set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/it6
mkdir -p $O
timeout -k 10 900 python -m pytest tests -q -m gpu -x > $O/pytest_gpu.log 2>&1 && \
for c in cfg5 cfg3 cfg4; do timeout -k 10 300 python bench.py --config $c --steps 10 --no-cpu-baseline > $O/$c.json 2> $O/$c.err || exit 1; done && \
timeout -k 10 300 python tools/ragged_diag.py > $O/diag.log 2>&1 && \
echo done
