#!/usr/bin/env bash
# Host AddressSanitizer + UBSan run of the native CSV parser (the only host C++
# on the data path).  Usage: tools/sanitize/run.sh [csv files...]
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
root="$(cd "$here/../.." && pwd)"
out="${TMPDIR:-/tmp}/har_csv_asan"
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
    -pthread "$here/csv_fuzz_main.cpp" "$root/csrc/host/csv_parser.cpp" -o "$out"
files=("$@")
if [ ${#files[@]} -eq 0 ] && [ -f "$root/data/wisdm_data.csv" ]; then files=("$root/data/wisdm_data.csv"); fi
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 "$out" "${files[@]}"
# ThreadSanitizer build (race detection for the multithreaded row split / merge)
g++ -std=c++17 -O1 -g -fsanitize=thread -pthread "$here/csv_fuzz_main.cpp" "$root/csrc/host/csv_parser.cpp" \
    -o "$out.tsan"
TSAN_OPTIONS=halt_on_error=1 "$out.tsan" "${files[@]}"
