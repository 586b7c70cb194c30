# Round 6: a parity fuzz campaign at the final tree (tooling): the batch fuzz
# (tests/test_gpu_fuzz.py, every entry point) over new seeds and many more
# rounds, and the in-launch tail fuzz (tests/test_gpu_tail.py::test_tail_fuzz)
# over many random uniform batches, each call bit-exact against the oracle.
# usage: gpurun -- 'bash tools/gpu_r6m.sh'
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6m
mkdir -p $O
P="python -u -m pytest -x -v -s -p no:cacheprovider --timeout 1500 --timeout-method thread"
TAIL_FUZZ_CASES=${TAIL_FUZZ_CASES:-4} timeout -k 10 300 $P tests/test_gpu_tail.py::test_tail_fuzz > $O/tail_check.log 2>&1 || exit $?
TAIL_FUZZ_CASES=${TF_CASES:-40} TAIL_FUZZ_SEED=${TF_SEED:-6} timeout -k 10 1200 $P tests/test_gpu_tail.py::test_tail_fuzz > $O/tail_fuzz_seed${TF_SEED:-6}.log 2>&1 || exit $?
for s in ${FUZZ_SEEDS:-1}; do
  FUZZ_ROUNDS=400 FUZZ_SEED=$s timeout -k 10 1500 $P tests/test_gpu_fuzz.py > $O/fuzz_seed$s.log 2>&1 || exit $?
done
tail -n 3 $O/*.log
