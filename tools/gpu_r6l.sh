# Round 6: the host runtime's sanitizer builds (tools/sanitize_host_runtime.sh,
# built in this container into build/san_asan and build/san_tsan) run on the
# GPU with every call on it.  usage: bash tools/gpu_r6l.sh
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r6l
mkdir -p $O/asan $O/tsan
export VAL_GPU_HOST_BATCH_MIN_BYTES=0 VAL_GPU_PROVIDER_MIN_BYTES=0
ASAN_OPTIONS="detect_leaks=0 log_path=$O/asan/san" UBSAN_OPTIONS="print_stacktrace=1 log_path=$O/asan/san" \
  timeout -k 10 600 build/san_asan/check 8 12 9 > $O/asan/check.out 2> $O/asan/check.err
rc=$?; echo "asan rc=$rc"; cat $O/asan/check.out; ls $O/asan
[ $rc -eq 0 ] || exit $rc
TSAN_OPTIONS="exitcode=0 log_path=$O/tsan/san" \
  timeout -k 10 600 build/san_tsan/check 4 6 9 > $O/tsan/check.out 2> $O/tsan/check.err
rc=$?; echo "tsan rc=$rc"; cat $O/tsan/check.out; ls $O/tsan | head
exit $rc
