"""Diagnostic: merge sorts (four-way passes) at several sizes against numpy; first mismatch."""
import importlib, os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
import torch
ls = importlib.import_module("radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd")
for lg in [int(x) for x in os.environ.get("LOG2NS", "17 18 19 20 21").split()] + [-1, -2]:
    n = (1 << lg) if lg > 0 else {-1: 300000, -2: 1234567}[lg]
    for dist, key in (("u32", "u32"), ("mod100", "u32"), ("sorted", "u32"), ("u32", "i32")):
        t = torch.empty(n, dtype=torch.int32, device="cuda")
        ls.fill(t, n, 0x5EED0002, dist)
        o = torch.empty_like(t)
        ws = torch.empty(ls.workspace_bytes(n, "merge"), dtype=torch.uint8, device="cuda")
        ls.sort_device(t, o, n, key=key, algo="merge", workspace=ws)
        torch.cuda.synchronize()
        vt = np.uint32 if key == "u32" else np.int32
        exp = np.sort(t.cpu().numpy().view(vt))
        got = o.cpu().numpy().view(vt)
        bad = np.nonzero(got != exp)[0]
        print(f"n={n} {dist} {key}: {'ok' if bad.size == 0 else f'{bad.size} wrong, first at {bad[0]} (got {got[bad[0]]}, want {exp[bad[0]]}), last at {bad[-1]}'}", flush=True)
