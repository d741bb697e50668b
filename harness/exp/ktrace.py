"""Print the last sort's kernel sequence from a rocprofv3 kernel trace: name, duration
and the idle gap before each launch (shows launch- vs bandwidth-bound passes)."""
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "labsort" in r["Kernel_Name"] or "k_" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 16
prev = None
for r in rows[-last:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f'{r["Kernel_Name"][:60]:60s} {(e - s) / 1e3:8.2f} us  gap {gap:6.2f} us  grid {r.get("Grid_Size", "")}')
    prev = e
