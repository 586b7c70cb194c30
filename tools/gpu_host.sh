set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/host; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python tools/host_inclusive.py > $O/host_inclusive.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; grep -v amdgpu.ids $O/host_inclusive.log; echo rc=$rc; exit $rc
