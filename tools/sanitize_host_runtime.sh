# Sanitizer runs of the library's host runtime (build container, CPU only):
# the whole library rebuilt with the host side instrumented (hipcc: each
# -fsanitize= after -Xarch_host, so device code is untouched; the C sources
# with the same clang), driven by oracle/host_runtime_check.c -- several
# threads of random batches through the CPU engine and its helper threads,
# verify, the *_host_multi and region CPU routes and the scalar hooks, every
# output against the oracle.
# usage: bash tools/sanitize_host_runtime.sh asan|tsan OUTDIR [THREADS ITERS SEED]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
MODE=${1:?asan|tsan}
O=${2:?outdir}
TH=${3:-4}; IT=${4:-6}; SEED=${5:-1}
mkdir -p "$O"
CLANG=/opt/rocm/llvm/bin/clang
case $MODE in
  asan) SAN="address,undefined"; HOSTSAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined" ;;
  tsan) SAN="thread"; HOSTSAN="-Xarch_host -fsanitize=thread" ;;
  *) echo "mode: asan|tsan" >&2; exit 2 ;;
esac
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -fPIC $HOSTSAN -I"$R/include" -I"$R/val_protocol_amd/csrc" \
    -c "$R/val_protocol_amd/csrc/val_crc32_hip.hip" -o "$O/hip.o"
for f in val_wire cpu_crc32 val_batch; do
  $CLANG -O1 -g -fPIC -std=gnu99 -fsanitize=$SAN -fno-omit-frame-pointer -I"$R/include" -I"$R/val_protocol_amd/csrc" \
      -c "$R/val_protocol_amd/csrc/$f.c" -o "$O/$f.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $HOSTSAN -o "$O/libval_san.so" "$O/hip.o" "$O/val_wire.o" \
    "$O/cpu_crc32.o" "$O/val_batch.o" -lpthread
$CLANG -O1 -g -std=gnu99 -fsanitize=$SAN -fno-omit-frame-pointer -I"$R/include" -I"$R/oracle" -o "$O/check" \
    "$R/oracle/host_runtime_check.c" "$R/oracle/crc32_oracle.c" "$O/libval_san.so" -Wl,-rpath,"$O" -lpthread
export ASAN_OPTIONS="detect_leaks=0 log_path=$O/san" UBSAN_OPTIONS="print_stacktrace=1 log_path=$O/san" \
       TSAN_OPTIONS="exitcode=0 log_path=$O/san"
: > "$O/stderr.txt"
"$O/check" "$TH" "$IT" "$SEED" 2>> "$O/stderr.txt"
cat "$O"/san.[0-9]* "$O/stderr.txt" > "$O/report.txt" 2>/dev/null || :
