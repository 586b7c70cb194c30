# HBM-traffic PMC passes only (cfg3, cfg3 verify, cfg5), each in its own
# rocprofv3 run, plus the provenance record (VAL_TREE = the commit, set by the
# caller): refreshes profiles/pmc_<cfg>.json after a library change without a
# whole round profile. Then: python tools/round_summary.py gpurun_out/round NN
# (the bench lines and traces of an earlier profile in that directory are kept).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/round
mkdir -p $O
echo "{\"tree\": \"${VAL_TREE:-unknown}\", \"box\": \"$(hostname)\", \"date\": \"$(date -u +%FT%TZ)\", \"lib_srchash\": \"$(cat $R/val_protocol_amd/libval_crc_hip.so.srchash)\"}" > $O/provenance.json
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o p -- python3 $R/tools/prof_target.py cfg3 3 > $O/pmc_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o p -- python3 $R/tools/prof_target.py cfg3 3 > $O/pmc_write.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_v -o p -- python3 $R/tools/prof_target.py cfg3 3 verify > $O/pmc_fetch_v.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch5 -o p -- python3 $R/tools/prof_target.py cfg5 3 > $O/pmc_fetch5.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write5 -o p -- python3 $R/tools/prof_target.py cfg5 3 > $O/pmc_write5.log 2>&1
echo "pmc rc=$?"
