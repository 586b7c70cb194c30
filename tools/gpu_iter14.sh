set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/it14
mkdir -p $O
timeout -k 10 900 python -m pytest tests -q -m gpu -x > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py build/libval_A.so build/libval_B.so u65532d u45000d u16400d > $O/ab.log 2>&1 && \
timeout -k 10 300 python bench.py --config cfg4 --no-cpu-baseline > $O/cfg4.json 2> $O/cfg4.err && \
SWEEP_LENGTHS=600,1100,2100,4200,8300,12000,16500,24000,33000,45000,49200,57000,65540 timeout -k 10 500 python tools/sweep_lengths.py > $O/sweep_len.log 2>&1 && echo done
