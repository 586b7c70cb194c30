set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/small; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o p -- python3 $R/tools/prof_small.py 20 w256:0:-1 w256:4:1 w256:16:1 w256:64:1 cfg2:0:-1 cfg2:2:1 cfg2:4:0 cfg2:4:1 cfg2:4:2 cfg2:8:1 cfg2:16:1 > $O/a.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/m5 -o p -- $R/bench/micro/mb5 > $O/mb5.log 2>&1
rc=$?; echo rc=$rc; exit $rc
