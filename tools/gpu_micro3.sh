set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/m3; mkdir -p $O
timeout -k 10 300 ./bench/micro/mb3 > $O/mb3.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace5 -o p -- python3 $R/tools/prof_target.py cfg5 5 > $O/trace5.log 2>&1
rc=$?; cat $O/mb3.log; echo rc=$rc; exit $rc
