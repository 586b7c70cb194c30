set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/it4
mkdir -p $O
timeout -k 10 900 python -m pytest tests -q -m gpu -x > $O/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> $O/pytest_gpu.log
for c in cfg5 cfg3 cfg4 cfg2; do timeout -k 10 300 python bench.py --config $c --steps 10 --no-cpu-baseline > $O/$c.json 2> $O/$c.err || exit 1; done
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace5 -o t -- python3 $GRAFT_REPO_ROOT/bench.py --config cfg5 --steps 5 --no-cpu-baseline > $O/trace5.log 2>&1
echo done
