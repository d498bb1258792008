#!/bin/bash
# Host-side sanitizer runs of the native runtime (engine, HTTP server, load generator) on the
# CPU backend: AddressSanitizer + UBSan, then ThreadSanitizer. No GPU needed; runs here or on a box.
#   bash tools/sanitize.sh [asan|tsan]...
set -u
cd "$(dirname "$0")/.."
OUT=build/sanitize
mkdir -p "$OUT"
SRC="csrc/tests/stress_host.cpp csrc/tests/kernel_stubs.cpp csrc/runtime/engine.cpp csrc/http/server.cpp csrc/http/json_body.cpp csrc/http/dispatch.cpp csrc/http/loadgen.cpp"
COMMON="--offload-arch=gfx950 -std=c++17 -O1 -g -fno-omit-frame-pointer -Icsrc -Icsrc/include -lpthread -ldl"
rc=0
for kind in ${*:-asan tsan}; do
  case $kind in
    asan) FLAGS="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined" ;;
    tsan) FLAGS="-Xarch_host -fsanitize=thread" ;;
    *) echo "unknown sanitizer $kind"; exit 2 ;;
  esac
  echo "== build $kind"
  /opt/rocm/bin/hipcc $FLAGS $COMMON $SRC -o "$OUT/stress_$kind" || { echo "build failed ($kind)"; exit 1; }
  echo "== run $kind"
  ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 \
    timeout -k 10 600 "$OUT/stress_$kind" || { echo "FAILED ($kind)"; rc=1; }
done
exit $rc
