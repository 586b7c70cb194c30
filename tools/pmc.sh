# PMC passes (separate rocprofv3 runs, --pmc only with kernel trace; no sys/runtime trace)
set -o pipefail
OUT=${1:-$GRAFT_REPO_ROOT/gpurun_out/pmc}
CFG=${2:-cfg3}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o t -- python3 $R/tools/prof_target.py $CFG 5 > $OUT/trace.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/p1 -o p -- python3 $R/tools/prof_target.py $CFG 3 > $OUT/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/p2 -o p -- python3 $R/tools/prof_target.py $CFG 3 > $OUT/p2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_INSTS_VMEM_RD --output-format csv -d $OUT/p3 -o p -- python3 $R/tools/prof_target.py $CFG 3 > $OUT/p3.log 2>&1
echo "pmc rc=$?"
