# Round-5 probe: ragged class lanes (VCRC_CLASS_LANES variants V1..V3) against
# the product (A), back to back, on the cfg5 mix, the class-2 mix and
# uniform short frames through the ragged path.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/g4; mkdir -p $O
timeout -k 10 400 python tools/ab_b2b.py build/libval_A.so build/libval_V1.so build/libval_V2.so build/libval_V3.so cfg5log c2 u1100 u3000 > $O/ab_lanes.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu $O/ab_lanes.log; exit $rc
