set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/ab_region.py build/ab/base.so build/ab/same.so build/ab/noev.so build/ab/noevhash.so > gpurun_out/ab_region2.log 2>&1 && \
timeout -k 10 300 python tools/ab_libs.py build/ab/base.so build/ab/noev.so cfg5log w256 > gpurun_out/ab_arena.log 2>&1
rc=$?
cat gpurun_out/ab_region2.log gpurun_out/ab_arena.log
exit $rc
