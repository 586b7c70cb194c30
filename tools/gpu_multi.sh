# Rehearse the N>1 bench path on a 1-GPU box: 2 ranks share cuda:0, gloo for the barrier/max.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/multi; mkdir -p $O
VAL_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench2.json 2> $O/bench2.err
rc=$?; cat $O/bench2.json; tail -3 $O/bench2.err; echo rc=$rc; exit $rc
