set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/it2
mkdir -p $O
timeout -k 10 900 python -m pytest tests -q -m gpu -x > $O/pytest_gpu.log 2>&1; echo "pytest rc=$?" >> $O/pytest_gpu.log
timeout -k 10 300 python bench.py --config cfg5 --steps 10 > $O/cfg5.json 2> $O/cfg5.err && \
timeout -k 10 300 python bench.py --config cfg5 --steps 10 --verify > $O/cfg5_verify.json 2> $O/cfg5_verify.err && \
timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline > $O/cfg3.json 2> $O/cfg3.err && \
timeout -k 10 300 python bench.py --config cfg2 --steps 100 --no-cpu-baseline > $O/cfg2.json 2> $O/cfg2.err
echo done
