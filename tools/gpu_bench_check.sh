# bench lines (cfg3 default, cfg2, cfg5) and a rocprofv3 kernel trace of the cfg3 bench command. Tooling only.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/bc; mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && \
timeout -k 10 600 python bench.py --config cfg2 --no-cpu-baseline --steps 200 > $O/bench_cfg2.json 2> $O/bench_cfg2.err && \
timeout -k 10 600 python bench.py --config cfg5 --no-cpu-baseline > $O/bench_cfg5.json 2> $O/bench_cfg5.err && \
timeout -k 10 600 python -u -m pytest tests/test_gpu_multiproc.py -x -q --timeout 300 --timeout-method thread > $O/pytest_multiproc.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o bench -- python3 $R/bench.py --no-cpu-baseline > $O/trace.log 2>&1
rc=$?; tail -2 $O/pytest_multiproc.log; for f in bench bench_cfg2 bench_cfg5; do tail -1 $O/$f.json | cut -c1-400; grep "per-step" $O/$f.err; done; echo rc=$rc; exit $rc
