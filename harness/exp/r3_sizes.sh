#!/bin/bash
# r3_sizes.sh -- size sweep of the final build: gathered radix (fused up to 2^20) vs merge
# at the AUTO crossover, uniform and three distributions
set -o pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd /tmp && export TMPDIR=/tmp
NS="65536 98304 131072 196608 262144 393216 524288 1048576"
echo "== u32"
NS="$NS" B2B=1 IMPLS="radix:gather merge" timeout -k 10 200 python3 "$R/harness/exp/small_n.py" || exit 1
for d in mod1000 sorted lowbits; do
  echo "== $d"
  DIST=$d PARAM=12 NS="65536 131072 262144 1048576" B2B=1 IMPLS="radix:gather merge" timeout -k 10 200 python3 "$R/harness/exp/small_n.py" || exit 1
done
