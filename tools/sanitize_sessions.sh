# Sanitizer runs of the batched drop-in (build container, CPU only):
# val_batch.c instrumented inside a copy of the product library (the HIP
# object is the one in build/), the reference sessions in
# oracle/provider_harness.c instrumented too.
#   tsan: ThreadSanitizer, four batched transfers at once (8 session threads
#         sharing the provider registry)
#   asan: AddressSanitizer + UndefinedBehaviorSanitizer (the CPU engine
#         cpu_crc32.c instrumented as well), one batched transfer at window 32
#         over a transport whose recv returns 1..3000 bytes (random per call),
#         then four at once
#   both: the round-6 fault runs (sendfail, oversize, stale recv_buffer calls)
# usage: bash tools/sanitize_sessions.sh tsan|asan OUTDIR   (needs /root/reference
# and a built library). Prints the harness's JSON lines; the sanitizers'
# reports go to OUTDIR/report.txt.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
REF=${REF:-/root/reference}
MODE=${1:?tsan|asan}
O=${2:?outdir}
mkdir -p "$O"
: > "$O/stderr.txt"
case $MODE in
  tsan) SAN="-fsanitize=thread"; CPU_O="$R/build/cpu_crc32.o" ;;
  asan) SAN="-fsanitize=address,undefined -fno-omit-frame-pointer"; CPU_O="$O/cpu.o"
        gcc -O1 -g -fPIC -std=gnu99 $SAN -I"$R/val_protocol_amd/csrc" -c "$R/val_protocol_amd/csrc/cpu_crc32.c" -o "$CPU_O" ;;
  *) echo "mode: tsan|asan" >&2; exit 2 ;;
esac
gcc -O1 -g -fPIC -std=c99 $SAN -I"$R/include" -c "$R/val_protocol_amd/csrc/val_batch.c" -o "$O/batch.o"
g++ -shared $SAN -o "$O/libval_san.so" "$R/build/val_crc32_hip.o" "$R/build/val_wire.o" "$CPU_O" "$O/batch.o" \
    -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -lpthread
gcc -O1 -g -std=gnu99 -w $SAN -DVAL_ENABLE_METRICS=1 -DVAL_LOG_LEVEL=0 -I"$REF/include" -I"$REF/src" \
    -I"$R/oracle" -o "$O/harness" "$R/oracle/provider_harness.c" "$REF/src/val_core.c" "$REF/src/val_wire.c" \
    "$REF/src/val_sender.c" "$REF/src/val_receiver.c" -ldl -lpthread
export TSAN_OPTIONS="exitcode=0 log_path=$O/san" ASAN_OPTIONS="detect_leaks=0 log_path=$O/san" \
       UBSAN_OPTIONS="print_stacktrace=1 log_path=$O/san"
if [ "$MODE" = asan ]; then
  VAL_HARNESS_PARTIAL=r3000 VAL_HARNESS_SEED=7 "$O/harness" "$O/libval_san.so" loopback-batched 1048576 4096 32 2>> "$O/stderr.txt" | tail -1
fi
# round 6: the batcher's fault contracts (a failed send in a window and the
# transfer after it, an oversize header and the transfer after it, stale
# recv_buffer calls against an armed answer)
VAL_HARNESS_MAX_TIMEOUT_MS=600 "$O/harness" "$O/libval_san.so" sendfail 1048576 1024 8 20 1 2>> "$O/stderr.txt" | tail -1
VAL_HARNESS_MAX_TIMEOUT_MS=600 "$O/harness" "$O/libval_san.so" oversize 1048576 1024 8 100 1 2>> "$O/stderr.txt" | tail -1
VAL_HARNESS_STALE_ARM=1 "$O/harness" "$O/libval_san.so" loopback-batched 1048576 1024 8 2>> "$O/stderr.txt" | tail -1
"$O/harness" "$O/libval_san.so" loopback-batched-par 2000000 4096 32 4 2>> "$O/stderr.txt" | tail -1
cat "$O"/san.[0-9]* "$O/stderr.txt" > "$O/report.txt" 2>/dev/null || :
