# rocprofv3 kernel trace of tools/prof_small.py over the given specs (name:G:PF).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/specs; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/t -o p -- python3 $R/tools/prof_small.py 10 "$@" > $O/a.log 2>&1
rc=$?; echo rc=$rc; exit $rc
