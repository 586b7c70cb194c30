# Round 6: the suite, a same-box A/B of the dynamic-tail rule change against
# the previous library (build/ab/libA.so = tools/build_rev.sh of 2eb74f2), and
# the driver's default bench line.  usage: gpurun -- 'bash tools/gpu_r6p.sh'
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6p
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -v -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/ab_b2b.py build/ab/libA.so val_protocol_amd/libval_crc_hip.so cfg3b cfg4d t65556 t32778 \
  u1100d u600d u2000d u4200d d262144x1100 d524288x1100 w131077x16400 w262150x4200 cfg2 cfg5log > $O/ab_final.log 2>&1 || exit 5
grep -v amdgpu.ids $O/ab_final.log | cut -c1-110
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 6
cat $O/bench.json | cut -c1-600
