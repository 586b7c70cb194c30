set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/m5; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/t -o p -- $R/bench/micro/mb5 > $O/mb5.log 2>&1
rc=$?; echo rc=$rc; exit $rc
