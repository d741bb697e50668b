"""Diagnostic: average launch time per timing class of a 2^28 sort (ALGO=radix: the
"histogram" and "onesweep" classes; ALGO=merge: "tile_sort" and "merge"), for A/B of
library builds whose results may be invalid (LABSORT_HS_DIAG_*, LABSORT_MG_DIAG_*
timing builds)."""
import importlib, json, os, sys
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
import torch
ls = importlib.import_module("radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd")
n = 1 << 28
d = torch.empty(n, dtype=torch.int32, device="cuda")
ls.fill(d, n, 0x5EED0003, os.environ.get("DIST", "u32"))
o = torch.empty_like(d)
algo = os.environ.get("ALGO", "radix")
classes = ("histogram", "onesweep") if algo == "radix" else ("tile_sort", "merge")
ws = torch.empty(ls.workspace_bytes(n, algo), dtype=torch.uint8, device="cuda")
for _ in range(3):
    ls.sort_device(d, o, n, algo=algo, workspace=ws)
torch.cuda.synchronize()
ls.timing_enable(True)
for _ in range(10):
    ls.sort_device(d, o, n, algo=algo, workspace=ws)
torch.cuda.synchronize()
row = {"lib": os.path.basename(os.environ.get("LABSORT_LIBRARY", "liblabsort.so")), "algo": algo,
       "ts_impl": os.environ.get("LABSORT_TS_IMPL", "")}
for c in classes:
    ms, cnt = ls.timing_read(c)
    row[c + "_ms"] = round(ms / max(cnt, 1), 4)
ls.timing_enable(False)
print(json.dumps(row))
