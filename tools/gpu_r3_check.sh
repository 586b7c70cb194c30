set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r3b; mkdir -p $O
lscpu > $O/lscpu.txt
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 --list-avail > $O/avail.txt 2>&1) || true
cd $R
timeout -k 10 300 python3 -u tools/provider_latency.py > $O/provider_latency.log 2>&1 && \
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "rc=$?"
tail -3 $O/pytest_gpu.log
