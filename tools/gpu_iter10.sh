set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/it11
mkdir -p $O
timeout -k 10 600 python -m pytest tests -q -m gpu -x > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py build/libval_A.so build/libval_B.so cfg5log cfg5 u57 u600 > $O/ab.log 2>&1 && \
timeout -k 10 300 python tools/ragged_diag.py > $O/diag.log 2>&1 && echo done
