#!/bin/bash
# harness/build.sh -- compile the reference's own benchmark drivers, UNCHANGED and
# straight from where they lie under /root/reference, against this repo's drop-in
# headers (include/lab.h, include/utils.h) and liblabsort.so.  This is the
# "main.cpp/performanceTest.cpp link unchanged" check of the north_star.
#
# main.cpp / performanceTest.cpp include "include/lab.h" relative to their own
# directory, so each is compiled through a symlink placed next to a symlink of
# our include/ in a scratch directory; nothing from the reference is copied.
# Outputs: harness/bin/sort, harness/bin/performaceTest (git-ignored; they travel
# to the GPU box with the snapshot and find liblabsort.so through an $ORIGIN rpath).
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
REPO="$(cd "$HERE/.." && pwd)"
REF="${LABSORT_REFERENCE:-/root/reference/Sord Radix y Merge}"
PKG="radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd"
if [ ! -f "$REF/main.cpp" ]; then
    echo "harness: reference sources not present ($REF); keeping prebuilt binaries" >&2
    exit 0
fi
SCRATCH="$(mktemp -d /tmp/labsort_harness.XXXXXX)"
trap 'rm -rf "$SCRATCH"' EXIT
ln -s "$REPO/include" "$SCRATCH/include"
ln -s "$REF/main.cpp" "$SCRATCH/main.cpp"
ln -s "$REF/performanceTest.cpp" "$SCRATCH/performanceTest.cpp"
mkdir -p "$HERE/bin"
# same flags as the reference Makefile:1-3 minus the nvcc-only ones
CXXFLAGS="-O3 -std=c++11"
LDFLAGS="-L$REPO/$PKG -llabsort -Wl,-rpath,\$ORIGIN/../../$PKG -lm -lpthread"
g++ $CXXFLAGS "$SCRATCH/main.cpp" -o "$HERE/bin/sort" $LDFLAGS
g++ $CXXFLAGS "$SCRATCH/performanceTest.cpp" -o "$HERE/bin/performaceTest" $LDFLAGS
echo "harness: built $HERE/bin/sort $HERE/bin/performaceTest"
