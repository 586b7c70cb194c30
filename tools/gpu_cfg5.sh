set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/cfg5
mkdir -p $O
for G in 0 4 8 16 32; do
  VAL_GPU_LANES_PER_FRAME=$G timeout -k 10 300 python bench.py --config cfg5 --steps 10 > $O/cfg5_G$G.json 2> $O/cfg5_G$G.err || exit 1
  VAL_GPU_LANES_PER_FRAME=$G timeout -k 10 300 python bench.py --config cfg5 --steps 10 --sort-frames > $O/cfg5_sorted_G$G.json 2> $O/cfg5_sorted_G$G.err || exit 1
done
timeout -k 10 300 python bench.py --config cfg5 --steps 10 --verify > $O/cfg5_verify.json 2> $O/cfg5_verify.err
echo done
