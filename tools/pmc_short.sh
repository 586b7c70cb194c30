# PMC passes (one rocprofv3 run per counter group, kernel trace only) over the
# A/B workloads named as arguments: instruction mix, waits, and L2->memory read
# requests by size (FETCH_SIZE attribution). Tooling only; writes gpurun_out/pmcs.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcs; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for W in "$@"; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$W/trace -o t -- python3 $R/tools/prof_wl.py $W 5 > $O/$W.trace.log 2>&1 && \
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD --output-format csv -d $O/$W/p1 -o p -- python3 $R/tools/prof_wl.py $W 3 > $O/$W.p1.log 2>&1 && \
  timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --output-format csv -d $O/$W/p2 -o p -- python3 $R/tools/prof_wl.py $W 3 > $O/$W.p2.log 2>&1 && \
  timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/$W/p3 -o p -- python3 $R/tools/prof_wl.py $W 3 > $O/$W.p3.log 2>&1 && \
  timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_DRAM_sum --output-format csv -d $O/$W/p4 -o p -- python3 $R/tools/prof_wl.py $W 3 > $O/$W.p4.log 2>&1 || { echo "failed at $W"; exit 1; }
  echo "done $W"
done
