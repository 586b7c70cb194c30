# Round 6 A/B: descriptor groups of 128-192 KiB with the one-word dynamic tail
# (B: -DVCRC_DYN_MIN_GROUP_DESC=131072) against static (A, the tree).
set -o pipefail
O=gpurun_out/r6i
mkdir -p $O
timeout -k 10 600 python tools/ab_libs.py build/libA_r6.so build/libD_r6.so cfg3d u16400d cfg4d t16390 cfg3b cfg3d > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 4; }
cat $O/ab.log
