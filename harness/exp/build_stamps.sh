#!/bin/bash
# Diagnostic build of liblabsort with onesweep phase stamps (-DOSP_STAMPS):
# harness/exp/liblabsort_stamps$SUFFIX.so.  Use with LABSORT_LIBRARY=<that path>.
# STAMPS= (empty) builds without stamps; EXTRA_FLAGS e.g. -DLABSORT_OSP_LBW=8.
set -e
R="$(cd "$(dirname "$0")/../.." && pwd)"
C="$R/radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/csrc"
B="$(mktemp -d)"
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 ${STAMPS--DOSP_STAMPS} ${EXTRA_FLAGS:-}"
SRCS=$(sed -n "s/^SRCS := //p" "$C/Makefile" | sed "s/\.hip//g")  # the product sources
for f in $SRCS; do /opt/rocm/bin/hipcc $F -c "$C/$f.hip" -o "$B/$f.o" & done; wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$R/harness/exp/liblabsort_stamps${SUFFIX:-}.so" "$B"/*.o -ldl -lpthread
rm -rf "$B"
