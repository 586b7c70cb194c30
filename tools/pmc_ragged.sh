set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/pmcr
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for m in strided57 ragged57 mix3 mix3aligned; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t_$m -o t -- python3 $GRAFT_REPO_ROOT/tools/prof_ragged.py $m > $O/t_$m.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD --output-format csv -d $O/p_$m -o p -- python3 $GRAFT_REPO_ROOT/tools/prof_ragged.py $m > $O/p_$m.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f_$m -o p -- python3 $GRAFT_REPO_ROOT/tools/prof_ragged.py $m > $O/f_$m.log 2>&1 || exit 1
done
echo done
