#!/bin/bash
# oracle_asan.sh -- the CPU tests that run the shared multi-GPU schedule (csrc/dist_plan.h,
# through oracle/dist_host.cpp) and the oracle under AddressSanitizer + UBSan (host code
# only, this container): builds a sanitized liboracle.so in a temp dir, swaps it in for the
# run, restores the normal build after.
set -e
R="$(cd "$(dirname "$0")/../.." && pwd)"
T=$(mktemp -d /tmp/oasan.XXXX)
F="-O1 -g -fPIC -fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined"
I="-I$R/include"
gcc $F -Wall -c "$R/oracle/labcu_restate.c" -o "$T/a.o"
g++ $F -Wall -fopenmp -std=c++17 $I -c "$R/oracle/cpu_sort.cpp" -o "$T/b.o"
g++ $F -Wall -fopenmp -std=c++17 $I -c "$R/oracle/dist_host.cpp" -o "$T/c.o"
g++ -shared -fopenmp -fsanitize=address,undefined -o "$T/liboracle.so" "$T"/*.o
cp "$R/oracle/liboracle.so" "$T/orig.so"
cp "$T/liboracle.so" "$R/oracle/liboracle.so"
trap 'cp "$T/orig.so" "$R/oracle/liboracle.so"; rm -rf "$T"' EXIT
cd "$R"
LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)" \
  ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  timeout 1200 python -m pytest tests/test_oracle.py tests/test_multi_plan.py tests/test_splitters.py \
  tests/test_dist_gloo.py -x -q -m "not gpu"
