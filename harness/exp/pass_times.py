"""Per-pass onesweep launch times from a rocprofv3 --kernel-trace CSV:
python pass_times.py <run_kernel_trace.csv> -- onesweep launches grouped by pass index
(the k-th onesweep launch after each histogram launch), plus the other labsort kernels."""
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
k, acc, other = -1, collections.defaultdict(list), collections.defaultdict(list)
for r in rows:
    nm = r["Kernel_Name"]
    dt = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    if "k_onesweep_p" in nm and k >= 0:
        acc[k].append(dt)
        k += 1
        continue
    if "k_hist_seg" in nm:
        k = 0
    if "labsort::" in nm:
        other[nm.split("(")[0].replace("labsort::", "")].append(dt)
for p in sorted(acc):
    v = sorted(acc[p])
    print(f"pass {p}: median {v[len(v)//2]:.4f} ms  min {v[0]:.4f}  (n={len(v)})")
for nm, v in sorted(other.items()):
    v = sorted(v)
    print(f"{nm[:40]:40s} median {v[len(v)//2]:.4f} ms (n={len(v)})")
