set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/sweep; mkdir -p $O
SWEEP_ROUNDS=${3:-1} SWEEP_COMBOS="$1" timeout -k 10 500 python tools/sweep_geometry.py $2 > $O/sweep.log 2>&1
rc=$?; grep -v amdgpu.ids $O/sweep.log; echo rc=$rc; exit $rc
