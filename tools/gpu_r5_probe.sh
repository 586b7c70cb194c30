# Round 5 ad-hoc probe: cfg3 at 8 vs 16 lanes per frame (bench.py, three
# alternations), then the session timings on the box's host (default
# thresholds, and everything forced onto the GPU).
set -o pipefail
mkdir -p gpurun_out/probe
for i in 1 2 3; do
for g in 8 16; do
VAL_GPU_LANES_PER_FRAME=$g timeout -k 10 200 python bench.py --no-cpu-baseline --no-host-inclusive --no-cfg4-strong --steps 20 > gpurun_out/probe/g$g.$i.json 2> gpurun_out/probe/g$g.$i.err || exit 3
python3 -c "import json; d=json.load(open('gpurun_out/probe/g$g.$i.json')); r=d['roofline']; print('G=$g', d['value'], r['kernel_ms'], r['read_roof'], r['frac_of_read_roof'], d['config']['lanes_per_frame'])"
done; done
timeout -k 10 400 python tools/session_timing.py 268435456 65536 64 3 > gpurun_out/probe/st_default.jsonl && \
timeout -k 10 300 python tools/session_timing.py 67108864 1024 64 3 > gpurun_out/probe/st_default_1024.jsonl && \
VAL_GPU_HOST_BATCH_MIN_BYTES=0 VAL_GPU_PROVIDER_MIN_BYTES=0 timeout -k 10 400 python tools/session_timing.py 268435456 65536 64 3 > gpurun_out/probe/st_gpu.jsonl
