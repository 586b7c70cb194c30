set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/it9
mkdir -p $O
timeout -k 10 600 python -m pytest tests -q -m gpu -x > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py build/libval_A.so build/libval_B.so cfg3 cfg3b cfg5 u57 > $O/ab.log 2>&1 && echo done
