# FETCH_SIZE (x2 = HBM read bytes on gfx950) and kernel time of one workload
# under several environment settings (e.g. forced lanes per frame), one
# rocprofv3 run per setting. Usage: pmc_variants.sh WORKLOAD "ENV=.. ENV2=.." ...
# Tooling only; writes gpurun_out/pmcv/<workload>_<i>/.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcv; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
W=$1; shift
i=0
for V in "$@"; do
  D=$O/${W}_$i; mkdir -p $D; echo "$V" > $D/env.txt
  ( export $V
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o t -- python3 $R/tools/prof_wl.py $W 5 > $D/trace.log 2>&1 && \
    timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/p3 -o p -- python3 $R/tools/prof_wl.py $W 3 > $D/p3.log 2>&1 ) || { echo "failed at $W $V"; exit 1; }
  echo "done $W [$V]"
  i=$((i+1))
done
