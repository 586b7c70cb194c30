# FETCH-derived traffic and kernel time of ragged-path and uniform-path workloads (product library). Tooling only.
set -o pipefail
R=$GRAFT_REPO_ROOT
for W in u16400 u16400d c2 cfg5log u1100 u1100d s4200; do
  bash $R/tools/pmc_variants.sh $W "VAL_GPU_X=0" || exit 1
done
