set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/ab_region.py build/ab/base.so build/ab/noatomic.so build/ab/nopow.so build/ab/hashonly.so > gpurun_out/ab_region.log 2>&1 && \
timeout -k 10 300 python bench.py --config cfg5 > gpurun_out/r2_bench_cfg5.log 2>&1 && \
timeout -k 10 120 python tools/timing_cfg2.py build/ab/timing.so cfg2 4 > gpurun_out/r2_timing_cfg2.log 2>&1 && \
timeout -k 10 120 python tools/timing_cfg2.py build/ab/timing.so cfg2 16 >> gpurun_out/r2_timing_cfg2.log 2>&1
rc=$?
cat gpurun_out/ab_region.log gpurun_out/r2_timing_cfg2.log; tail -c 1200 gpurun_out/r2_bench_cfg5.log
[ $rc -eq 0 ] || exit $rc
for m in 0 1 2; do timeout -k 10 120 ./bench/micro/repro_pageable $m 71680 3000 >> gpurun_out/r2_repro.log 2>&1 || exit 3; done
timeout -k 10 120 ./bench/micro/repro_pageable 0 1048576 1000 >> gpurun_out/r2_repro.log 2>&1
cat gpurun_out/r2_repro.log
