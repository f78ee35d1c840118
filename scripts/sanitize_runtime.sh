#!/bin/bash
# Build and run the native host-runtime self-test three times: plain (-O2), under ThreadSanitizer (the
# multi-threaded line packing) and under AddressSanitizer + UndefinedBehaviorSanitizer (host-side sanitizer build; GPU ASan / xnack+ is not
# available on the MI355X pool, so kernels are checked by numerics tests + in-kernel asserts).
# Sources: csrc/runtime/{json,safetensors,tokenizer,dataset,power_monitor} -- everything in the
# runtime that does not need the HIP runtime.  Usage: scripts/sanitize_runtime.sh [outdir]
set -euo pipefail
here="$(cd "$(dirname "$0")/.." && pwd)"
csrc="$here/mobilefinetuner_amd/csrc"
out="${1:-$here/build/selftest}"
mkdir -p "$out"
srcs=("$csrc/tests/runtime_selftest.cpp" "$csrc/runtime/safetensors.cpp" "$csrc/runtime/tokenizer.cpp"
      "$csrc/runtime/dataset.cpp" "$csrc/runtime/power_monitor.cpp")
CXX="${CXX:-g++}"
"$CXX" -std=c++17 -O2 -g -Wall -Wextra -Wno-unused-parameter -I"$csrc" "${srcs[@]}" -lpthread -o "$out/runtime_selftest"
"$CXX" -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
  -I"$csrc" "${srcs[@]}" -lpthread -o "$out/runtime_selftest_asan"
"$CXX" -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=thread -I"$csrc" "${srcs[@]}" -lpthread \
  -o "$out/runtime_selftest_tsan"
"$out/runtime_selftest"
TSAN_OPTIONS=halt_on_error=1 "$out/runtime_selftest_tsan"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=0 UBSAN_OPTIONS=print_stacktrace=1 "$out/runtime_selftest_asan"
echo "sanitized runtime selftest OK"
