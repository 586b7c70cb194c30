# FETCH_SIZE passes for cfg3 TX with and without header_crc (over-fetch diagnosis).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/fetch; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/hdr -o p -- python3 $R/tools/prof_target.py cfg3 3 > $O/hdr.log 2>&1 && \
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/nohdr -o p -- python3 $R/tools/prof_target.py cfg3 3 nohdr > $O/nohdr.log 2>&1
rc=$?; echo rc=$rc; exit $rc
