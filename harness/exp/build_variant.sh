#!/bin/bash
# build_variant.sh NAME "-DFLAG=.. ..." -- a diagnostic liblabsort build with extra
# defines into harness/exp/libs/liblabsort_NAME.so (select with LABSORT_LIBRARY)
set -e
HERE="$(cd "$(dirname "$0")" && pwd)"
C="$HERE/../../radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd/csrc"
mkdir -p "$HERE/libs" "/tmp/lsv_$1"
pids=()
SRCS=$(sed -n "s/^SRCS := //p" "$C/Makefile" | sed "s/\.hip//g")  # the product sources
for f in $SRCS; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -w $2 -c "$C/$f.hip" -o "/tmp/lsv_$1/$f.o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p || { echo "compile failed ($1)"; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$HERE/libs/liblabsort_$1.so" /tmp/lsv_$1/*.o -ldl -lpthread
echo "built harness/exp/libs/liblabsort_$1.so"
