# LDS / VALU / wait counters of the frames kernel for cfg2 and cfg3 (one PMC
# pass per rocprofv3 run; tooling only). Output under gpurun_out/pmc2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/pmc2
mkdir -p $O
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/sq_cfg2 -o p -- python3 $R/tools/prof_target.py cfg2 20 > $O/sq_cfg2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/sq_cfg3 -o p -- python3 $R/tools/prof_target.py cfg3 3 > $O/sq_cfg3.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY --output-format csv -d $O/act_cfg2 -o p -- python3 $R/tools/prof_target.py cfg2 20 > $O/act_cfg2.log 2>&1
echo "pmc_lds rc=$?"
