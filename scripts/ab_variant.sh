#!/bin/bash
# Build the working tree's library with extra compile flags into ab/<name>.so (same-box A/B of
# compile-time variants):   scripts/ab_variant.sh <name> "-DRT_GEN_WREG=4 -DRT_GEN_XREG=1"
set -e
name=$1; flags=$2
root=$(git rev-parse --show-toplevel)
tmp=$(mktemp -d)
cp -r "$root/include" "$tmp/"
mkdir -p "$tmp/ray-tracing-c_amd"
cp -r "$root/ray-tracing-c_amd/csrc" "$root/ray-tracing-c_amd/host" "$root/ray-tracing-c_amd/Makefile" "$tmp/ray-tracing-c_amd/"
make -C "$tmp/ray-tracing-c_amd" -j8 librtc_amd.so EXTRA_HIPFLAGS="$flags" > /dev/null
mkdir -p "$root/ab"
cp "$tmp/ray-tracing-c_amd/librtc_amd.so" "$root/ab/$name.so"
rm -rf "$tmp"
echo "ab/$name.so ($flags)"
