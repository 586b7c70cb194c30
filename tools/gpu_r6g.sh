# Round 6 probe: cfg3 frame layouts against 128-B lines (tools/layout_probe.py).
set -o pipefail
O=gpurun_out/r6g
mkdir -p $O
timeout -k 10 400 python tools/layout_probe.py > $O/layout.jsonl 2> $O/layout.err || { tail -20 $O/layout.err; exit 4; }
cat $O/layout.jsonl
