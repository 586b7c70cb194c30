# Traffic/time of u1100d and cfg3b under forced geometries and kernel switches (tools/pmc_variants.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/pmc_variants.sh u1100d "VAL_GPU_X=0" "VAL_GPU_CARRY=0" "VAL_GPU_LANES_PER_FRAME=2" "VAL_GPU_LANES_PER_FRAME=8" "VAL_GPU_LANES_PER_FRAME=16" "VAL_GPU_DYNAMIC_TAIL=0" && \
bash $R/tools/pmc_variants.sh cfg3b "VAL_GPU_X=0" "VAL_GPU_LANES_PER_FRAME=16" "VAL_GPU_LANES_PER_FRAME=4" "VAL_GPU_DYNAMIC_TAIL=0"
