# Round 6 probe: strided against descriptor mode on uniform batches (tools/desc_probe.py).
set -o pipefail
O=gpurun_out/r6h
mkdir -p $O
timeout -k 10 400 python tools/desc_probe.py > $O/desc.jsonl 2> $O/desc.err || { tail -20 $O/desc.err; exit 4; }
cat $O/desc.jsonl
