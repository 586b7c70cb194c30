# PMC + kernel trace of the ragged path (tools/prof_ragged.py), current build
# and optionally an older build for an A/B: bash tools/pmc_ragged.sh [OLD_LIB]
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/pmcr
mkdir -p $O
OLD=${1:+$GRAFT_REPO_ROOT/$1}
cd /tmp && export TMPDIR=/tmp
run() {  # tag mode [lib]
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_$1 -o t -- python3 $GRAFT_REPO_ROOT/tools/prof_ragged.py $2 $3 > $O/t_$1.log 2>&1 || return 1
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD --output-format csv -d $O/p_$1 -o p -- python3 $GRAFT_REPO_ROOT/tools/prof_ragged.py $2 $3 > $O/p_$1.log 2>&1 || return 1
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$1 -o p -- python3 $GRAFT_REPO_ROOT/tools/prof_ragged.py $2 $3 > $O/f_$1.log 2>&1 || return 1
}
for m in strided57 ragged57 mix3 mix3aligned; do run $m $m || exit 1; done
if [ -n "$OLD" ]; then for m in mix3 mix3aligned; do run old_$m $m $OLD || exit 1; done; fi
python3 $GRAFT_REPO_ROOT/tools/pmc_ragged_summary.py $O > $O/summary.txt && cat $O/summary.txt && echo done
