# Round-5 probe: the driver's default 8-GPU bench invocation (cfg3 + cfg4_strong
# + host_inclusive on rank 0) rehearsed as 8 gloo ranks on one GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/g8; mkdir -p $O
VAL_BENCH_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --steps 3 --warmup 1 > $O/bench8.json 2> $O/bench8.err
rc=$?; echo "rc=$rc"; tail -c 3000 $O/bench8.json; tail -5 $O/bench8.err; exit $rc
