#!/usr/bin/env bash
# Host ASan + UBSan build of every HIP kernel source's launcher code (device code compiled as usual
# for gfx950; the sanitizers apply to the host side only: -Xarch_host), linked with guards_main.cpp,
# which drives the launch-contract guards with bad arguments.  Needs no GPU.
#   usage: tools/sanitize/guards.sh [jobs]
set -euo pipefail
here="$(cd "$(dirname "$0")" && pwd)"
root="$(cd "$here/../.." && pwd)"
out="${TMPDIR:-/tmp}/har_guards"
mkdir -p "$out"
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
san=(-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined
     -Xarch_host -fno-omit-frame-pointer)
flags=(-O2 -std=c++17 --offload-arch=gfx950 -I "$root/csrc" -Wno-unused-result -Wno-unused-variable)
jobs="${1:-8}"
objs=()
pids=()
for src in "$root"/csrc/kernels/*.hip; do
  obj="$out/$(basename "$src").o"
  objs+=("$obj")
  "$HIPCC" "${flags[@]}" "${san[@]}" -x hip -munsafe-fp-atomics -c "$src" -o "$obj" &
  pids+=($!)
  if [ "${#pids[@]}" -ge "$jobs" ]; then wait "${pids[0]}"; pids=("${pids[@]:1}"); fi
done
for p in "${pids[@]}"; do wait "$p"; done
"$HIPCC" "${flags[@]}" "${san[@]}" -x hip -c "$here/guards_main.cpp" -o "$out/guards_main.o"
"$HIPCC" --offload-arch=gfx950 -fsanitize=address,undefined -fno-gpu-sanitize -o "$out/guards" "$out/guards_main.o" "${objs[@]}"
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 "$out/guards"
