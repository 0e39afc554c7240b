#!/bin/bash
# Build librtc_amd.so of a git revision into ab/<name>.so (same-box A/B: RTC_LIB=ab/<name>.so).
#   scripts/ab_build.sh <rev> <name>
set -e
rev=$1; name=$2
root=$(git rev-parse --show-toplevel)
tmp=$(mktemp -d)
git -C "$root" worktree add -q --detach "$tmp" "$rev"
make -C "$tmp/ray-tracing-c_amd" -j8 librtc_amd.so > /dev/null
mkdir -p "$root/ab"
cp "$tmp/ray-tracing-c_amd/librtc_amd.so" "$root/ab/$name.so"
git -C "$root" worktree remove --force "$tmp"
echo "ab/$name.so from $(git -C "$root" rev-parse --short "$rev")"
