#!/bin/bash
# Build the native extension of another commit into ab/<name>/_har_native.so (for tools/sessions/gpu_ab.sh):
#   bash tools/ab_build.sh <commit> <name>
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
WT="/tmp/har_ab_$2"
rm -rf "$WT"; git -C "$ROOT" worktree prune
git -C "$ROOT" worktree add --detach "$WT" "$1" > /dev/null
python3 "$WT/tools/build_native.py" > "/tmp/har_ab_$2.log" 2>&1
mkdir -p "$ROOT/ab/$2"
cp "$WT/activity-recognition-using-apache-spark_amd/_har_native.so" "$ROOT/ab/$2/_har_native.so"
git -C "$ROOT" worktree remove --force "$WT"
echo "ab/$2/_har_native.so <- $(git -C "$ROOT" rev-parse --short "$1")"
