#!/bin/bash
# Per-kernel register / scratch / occupancy summary of the gfx950 device code (no GPU needed).
#   scripts/kres.sh [out.s]     (asm also written to out.s, default /tmp/rt_kernel.s)
set -e
cd "$(dirname "$0")/../ray-tracing-c_amd"
OUT=${1:-/tmp/rt_kernel.s}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fno-fast-math -munsafe-fp-atomics -fno-slp-vectorize -std=c++17 -I../include $KRES_FLAGS \
  -S --offload-device-only -Rpass-analysis=kernel-resource-usage csrc/rt_kernel.hip -o "$OUT" 2>&1 |
  awk '/Function Name:/ {name=$NF; sub(/\[.*$/,"",name)} /Function Name/ {split($0,a,"Function Name: "); split(a[2],b," "); name=b[1]}
       /VGPRs:/ && !/AGPR/ {split($0,a,"VGPRs: "); split(a[2],b," "); v=b[1]}
       /ScratchSize/ {split($0,a,"lane\\]: "); split(a[2],b," "); s=b[1]}
       /Occupancy/ {split($0,a,"Occupancy \\[waves/SIMD\\]: "); split(a[2],b," "); printf "%-60s vgpr=%-4s scratch=%-5s occ=%s\n", name, v, s, b[1]}'
