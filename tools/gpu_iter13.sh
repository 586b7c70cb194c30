set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/it13
mkdir -p $O
L=$GRAFT_REPO_ROOT/val_protocol_amd/libval_crc_hip.so
timeout -k 10 300 python tools/ab_libs.py $L $L c2 c2a u16400 u16401 u16400d u16401d > $O/ab.log 2>&1 && \
SWEEP_LENGTHS=600,1100,2100,4200,8300,12000,16500,24000,33000,45000,49200,57000,65540 timeout -k 10 500 python tools/sweep_lengths.py > $O/sweep_len.log 2>&1 && echo done
