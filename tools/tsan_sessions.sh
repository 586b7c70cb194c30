# ThreadSanitizer run of the batched drop-in (build container, CPU only):
# val_batch.c instrumented inside a copy of the product library, the
# reference sessions in oracle/provider_harness.c instrumented too, four
# batched transfers at once (8 session threads sharing the provider registry).
# usage: bash tools/tsan_sessions.sh OUTDIR   (needs /root/reference and a built
# library: the HIP object is the one in build/). Prints the harness's JSON
# line; ThreadSanitizer reports go to OUTDIR/tsan.txt.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
REF=${REF:-/root/reference}
O=${1:?outdir}
mkdir -p "$O"
gcc -O1 -g -fPIC -std=c99 -fsanitize=thread -I"$R/include" -c "$R/val_protocol_amd/csrc/val_batch.c" -o "$O/batch.o"
g++ -shared -fsanitize=thread -o "$O/libval_tsan.so" "$R/build/val_crc32_hip.o" "$R/build/val_wire.o" \
    "$R/build/cpu_crc32.o" "$O/batch.o" -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib -lpthread
gcc -O1 -g -std=gnu99 -w -fsanitize=thread -DVAL_ENABLE_METRICS=1 -DVAL_LOG_LEVEL=0 -I"$REF/include" -I"$REF/src" \
    -I"$R/oracle" -o "$O/harness" "$R/oracle/provider_harness.c" "$REF/src/val_core.c" "$REF/src/val_wire.c" \
    "$REF/src/val_sender.c" "$REF/src/val_receiver.c" -ldl -lpthread
TSAN_OPTIONS="exitcode=0 log_path=$O/tsan" "$O/harness" "$O/libval_tsan.so" loopback-batched-par 2000000 4096 32 4
cat "$O"/tsan.[0-9]* > "$O/tsan.txt" 2>/dev/null || : > "$O/tsan.txt"
