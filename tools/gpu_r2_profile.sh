# Round-2 measurement call: the round profile (tests, smoke, bench lines,
# host-inclusive, rocprofv3 kernel traces and PMC passes) plus the multi-rank
# rehearsal of bench.py on one GPU (gloo).
bash tools/gpu_round_profile.sh && bash tools/gpu_multi.sh
