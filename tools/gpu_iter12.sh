set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/it12
mkdir -p $O
timeout -k 10 600 python -m pytest tests -q -m gpu -x > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py build/libval_A.so build/libval_B.so cfg5log cfg5 u600 > $O/ab.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tA -o t -- python3 $GRAFT_REPO_ROOT/tools/prof_ab.py u600 $GRAFT_REPO_ROOT/build/libval_A.so > $O/tA.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tB -o t -- python3 $GRAFT_REPO_ROOT/tools/prof_ab.py u600 > $O/tB.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t5 -o t -- python3 $GRAFT_REPO_ROOT/tools/prof_ab.py cfg5log > $O/t5.log 2>&1 && echo done
