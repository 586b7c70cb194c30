# f1/f2 call-site batching, end to end: reference per-frame TX/RX vs the
# batched GPU window path (oracle/_ref/provider_harness windowbench).
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/wb; mkdir -p $O
: > $O/windowbench.jsonl
for mtu in 1024 8192 65536; do for W in 16 64 256 1024 4096; do
  timeout -k 5 120 ./oracle/_ref/provider_harness val_protocol_amd/libval_crc_hip.so windowbench $W $mtu 7 >> $O/windowbench.jsonl || exit 1
done; done
cat $O/windowbench.jsonl
