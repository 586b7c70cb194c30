# FETCH_SIZE passes (one rocprofv3 run per variant, kernel trace + one counter)
# over u1100d, u600d and s1100 with the automatic rings, VAL_GPU_PREFETCH=1,
# the same on a -DVCRC_ILV16=0 build (build/libval_C.so) and VAL_GPU_PREFETCH=0.
# Tooling only; writes gpurun_out/pmcab (summary: profiles/r04_pmc_fetch_prefetch_variants.txt).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcab; mkdir -p $O; cd /tmp && export TMPDIR=/tmp
run() { tag=$1; shift; env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/$tag -o p -- python3 $R/tools/prof_wl.py $W 3 > $O/$tag.log 2>&1; }
for W in u1100d u600d s1100; do
  run ${W}_ring X=1 && run ${W}_pf1 VAL_GPU_PREFETCH=1 && run ${W}_pf1_noilv VAL_GPU_PREFETCH=1 PROF_LIB=$R/build/libval_C.so && run ${W}_pf0 VAL_GPU_PREFETCH=0 || exit 1
done
echo ok
