# Round 6 final: A/B of the descriptor dynamic-tail rule (A = previous tree,
# B = this tree), then the round-end profile of this tree.
set -o pipefail
O=gpurun_out/r6j
mkdir -p $O
timeout -k 10 600 python tools/ab_libs.py build/libA_r6.so val_protocol_amd/libval_crc_hip.so cfg3d u16400d cfg3b cfg4d cfg3d > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 4; }
cat $O/ab.log
bash tools/gpu_round_profile.sh
