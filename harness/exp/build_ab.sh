#!/bin/bash
# build_ab.sh NAME [REV] [make args...] -- build liblabsort from git revision REV (default HEAD)
# into harness/bin/ab/liblabsort_NAME.so, for same-box A/B runs against the working tree
set -e
R="$(cd "$(dirname "$0")/../.." && pwd)"
NAME=$1; REV=${2:-HEAD}; shift 2 || shift $#
T=$(mktemp -d /tmp/abuild.XXXX)
PKG=radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd
mkdir -p "$T/$PKG" "$R/harness/bin/ab"
git -C "$R" archive "$REV" "$PKG/csrc" include | tar -x -C "$T"
make -s -j8 -C "$T/$PKG/csrc" OUT="$R/harness/bin/ab/liblabsort_$NAME.so" "$@"
rm -rf "$T"
echo "built harness/bin/ab/liblabsort_$NAME.so from $REV"
