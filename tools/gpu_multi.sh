# Rehearse the N>1 bench path on a 1-GPU box: ranks share cuda:0, gloo for the barrier/max.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/multi; mkdir -p $O
VAL_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench2.json 2> $O/bench2.err && \
VAL_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 4 --config cfg4 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench4_cfg4.json 2> $O/bench4_cfg4.err && \
timeout -k 10 600 python bench.py --config cfg4 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench1_cfg4.json 2> $O/bench1_cfg4.err
rc=$?; cat $O/bench2.json $O/bench4_cfg4.json $O/bench1_cfg4.json; tail -3 $O/bench4_cfg4.err; echo rc=$rc; exit $rc
