# Memory-pipeline counters of the CRC kernel for tools/prof_ab.py workloads.
# usage: bash tools/pmc_mem.sh OUTDIR TAG:WORKLOAD[:LIB] ...
set -o pipefail
O=$GRAFT_REPO_ROOT/$1; shift
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
# at most two TA / TCP counters per pass (more fails with error 38 on gfx950)
P1="TA_TA_BUSY_sum TA_DATA_STALLED_BY_TC_CYCLES_sum"
P2="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum"
P3="TCP_UTCL1_TRANSLATION_MISS_sum TCP_PENDING_STALL_CYCLES_sum"
P4="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P5="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH"
for spec in "$@"; do
  IFS=: read tag wl lib <<< "$spec"
  L=${lib:+$GRAFT_REPO_ROOT/$lib}
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_$tag -o t -- python3 $GRAFT_REPO_ROOT/tools/prof_ab.py $wl $L > $O/t_$tag.log 2>&1 || exit 1
  i=0
  for P in "$P1" "$P2" "$P3" "$P4" "$P5"; do
    i=$((i+1))
    timeout -k 10 200 rocprofv3 --pmc $P --output-format csv -d $O/p${i}_$tag -o p -- python3 $GRAFT_REPO_ROOT/tools/prof_ab.py $wl $L > $O/p${i}_$tag.log 2>&1 || exit 1
  done
done
python3 $GRAFT_REPO_ROOT/tools/pmc_mem_summary.py $O > $O/summary.txt && cat $O/summary.txt
