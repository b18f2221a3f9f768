#!/bin/bash
# CPU sanitizer runs of the host-side code (VERDICT r02
# item 9).  No GPU: the library's host paths (host builds, serialize /
# deserialize validation, key-stream staging, CRC, concurrent host calls) and
# the oracle's multithreaded builds.
#   1. the library with -fsanitize=address,undefined on its HOST code (each
#      -fsanitize= after -Xarch_host: the device code is not instrumented),
#      driven by tests/cpp/host_sanitize.cpp and the C++ mirror of the
#      reference's bloom tests (tests/cpp/bloom_tests.cpp, host mode);
#   2. the same with -fsanitize=thread;
#   3. the oracle's threaded builds (oracle_bloom_build_*_mt) with
#      -fsanitize=thread, and its single-thread code with address,undefined.
# Usage: tools/sanitize.sh [outdir]   (log: <outdir>/sanitize.log)
set -u
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-$ROOT/storage-engine_amd/build/san}
mkdir -p "$OUT"
LOG=$OUT/sanitize.log
: > "$LOG"
HIPCC=/opt/rocm/bin/hipcc
CLANG=/opt/rocm/llvm/bin/clang++
CLANGC=/opt/rocm/llvm/bin/clang
SRCS="bloom_build bloom_probe capi multi stream crc32"
fails=0
run() {  # name, command...
  local name=$1; shift
  echo "== $name" | tee -a "$LOG"
  if "$@" >> "$LOG" 2>&1; then echo "   ok" | tee -a "$LOG"; else echo "   FAILED ($?)" | tee -a "$LOG"; fails=$((fails + 1)); fi
}
lib() {  # variant, host sanitizer flags...
  local v=$1; shift
  local flags=""
  for f in "$@"; do flags="$flags -Xarch_host $f"; done
  mkdir -p "$OUT/$v"
  for s in $SRCS; do
    $HIPCC -O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-value $flags \
      -Xarch_host -fno-omit-frame-pointer -c "$ROOT/storage-engine_amd/csrc/$s.hip" -o "$OUT/$v/$s.o" &
  done
  wait
  $HIPCC -shared -fPIC --offload-arch=gfx950 -o "$OUT/$v/liblsmbloom.so" $(for s in $SRCS; do echo "$OUT/$v/$s.o"; done)
}
drivers() {  # variant, sanitizer flags
  local v=$1 f=$2
  $CLANG -std=c++17 -O1 -g $f -fno-omit-frame-pointer -o "$OUT/$v/host_sanitize" "$ROOT/tests/cpp/host_sanitize.cpp" \
    -L"$OUT/$v" -llsmbloom -Wl,-rpath,"$OUT/$v" -lpthread
  $CLANG -std=c++17 -O1 -g $f -fno-omit-frame-pointer -I"$ROOT/storage-engine_amd" -o "$OUT/$v/bloom_tests" \
    "$ROOT/tests/cpp/bloom_tests.cpp" -L"$OUT/$v" -llsmbloom -Wl,-rpath,"$OUT/$v" -lpthread
}
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1

run "build library, host code -fsanitize=address,undefined" lib asan -fsanitize=address -fsanitize=undefined \
    -fno-sanitize-recover=undefined
run "build drivers (asan, ubsan)" drivers asan "-fsanitize=address,undefined -fno-sanitize-recover=undefined"
run "host_sanitize under asan+ubsan" "$OUT/asan/host_sanitize"
run "bloom_tests (C++ mirror, host mode) under asan+ubsan" "$OUT/asan/bloom_tests"
run "build library, host code -fsanitize=thread" lib tsan -fsanitize=thread
run "build drivers (tsan)" drivers tsan "-fsanitize=thread"
run "host_sanitize under tsan" "$OUT/tsan/host_sanitize"
run "bloom_tests (C++ mirror, host mode) under tsan" "$OUT/tsan/bloom_tests"
run "build oracle + threaded driver (tsan)" $CLANGC -O1 -g -std=c11 -D_GNU_SOURCE -fsanitize=thread -o "$OUT/oracle_mt_tsan" \
    "$ROOT/oracle/bloom_oracle.c" "$ROOT/tests/cpp/oracle_mt_tsan.c" -lm -lpthread
run "oracle threaded builds under tsan" "$OUT/oracle_mt_tsan"
run "build oracle + threaded driver (asan, ubsan)" $CLANGC -O1 -g -std=c11 -D_GNU_SOURCE -fsanitize=address,undefined \
    -fno-sanitize-recover=undefined -o "$OUT/oracle_mt_asan" "$ROOT/oracle/bloom_oracle.c" "$ROOT/tests/cpp/oracle_mt_tsan.c" -lm -lpthread
run "oracle builds under asan+ubsan" "$OUT/oracle_mt_asan"
echo "sanitize: $fails failure(s); log $LOG" | tee -a "$LOG"
exit $fails
