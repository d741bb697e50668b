"""Diagnostic: average k_hist_seg (timing class "histogram") and onesweep pass times of
the 2^28 radix sort, for A/B of library builds whose results may be invalid
(LABSORT_HS_DIAG_* timing builds)."""
import importlib, json, os, sys
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
import torch
ls = importlib.import_module("radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd")
n = 1 << 28
d = torch.empty(n, dtype=torch.int32, device="cuda")
ls.fill(d, n, 0x5EED0003, os.environ.get("DIST", "u32"))
o = torch.empty_like(d)
ws = torch.empty(ls.workspace_bytes(n, "radix"), dtype=torch.uint8, device="cuda")
for _ in range(3):
    ls.sort_device(d, o, n, algo="radix", workspace=ws)
torch.cuda.synchronize()
ls.timing_enable(True)
for _ in range(10):
    ls.sort_device(d, o, n, algo="radix", workspace=ws)
torch.cuda.synchronize()
h_ms, h_cnt = ls.timing_read("histogram")
p_ms, p_cnt = ls.timing_read("onesweep")
ls.timing_enable(False)
print(json.dumps({"lib": os.path.basename(os.environ.get("LABSORT_LIBRARY", "liblabsort.so")),
                  "hist_ms": round(h_ms / max(h_cnt, 1), 4), "pass_ms": round(p_ms / max(p_cnt, 1), 4)}))
