#!/bin/bash
# r6: the default bench line's radix and merge legs at 2^28 for each key distribution in DISTS
# (bench.py --dist; every output is verified by the bench itself), one summary line each.
set -e
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
O="$R/gpurun_out"; mkdir -p "$O"; cd "$R"
for d in ${DISTS:-u32 u31 mod1000 mod100 sorted reversed lowbits const}; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --no-host-path --dist $d > "$O/dist_$d.json" 2> "$O/dist_$d.err"
  python3 - "$O/dist_$d.json" "$d" <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
m = b.get("merge", {})
print(f"{sys.argv[2]:9s} radix {b['ms_per_step']:.4f} ms ({b['value'] / 1e3:.1f} Gkeys/s, verified: {b['verified'][:20]})  "
      f"merge {m.get('ms_per_step', float('nan')):.4f} ms ({m.get('value', 0) / 1e3:.1f} Gkeys/s)  "
      f"pairs {b.get('pairs', {}).get('ms_per_step', float('nan')):.4f} ms")
PY
done
