set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/m4; mkdir -p $O
timeout -k 10 300 ./bench/micro/mb4 > $O/mb4.log 2>&1
rc=$?; cat $O/mb4.log; echo rc=$rc; exit $rc
