# K4 region latency: events + host wall, then the same under rocprofv3 kernel trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python tools/region_latency.py > gpurun_out/r2_region.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_region -o region -- python3 tools/region_latency.py > gpurun_out/r2_region_prof.log 2>&1
rc=$?
cat gpurun_out/r2_region.log
find gpurun_out/prof_region -name "*kernel_stats.csv" | head -1 | xargs cat | cut -d, -f1-8 | head -12
exit $rc
