"""Diagnostic: merge sort of 2^18 sorted keys; dump the four-way pass's boundary table and
samples from the workspace and check them against numpy."""
import importlib, os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
import torch
ls = importlib.import_module("radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd")
n = 1 << int(os.environ.get("LOG2N", "18"))
dist = os.environ.get("DIST", "sorted")
t = torch.empty(n, dtype=torch.int32, device="cuda")
ls.fill(t, n, 0x5EED0002, dist)
o = torch.empty_like(t)
ws = torch.zeros(ls.workspace_bytes(n, "merge"), dtype=torch.uint8, device="cuda")
ls.sort_device(t, o, n, algo="merge", workspace=ws)
torch.cuda.synchronize()
al = lambda x: (x + 255) // 256 * 256
off_part = al(n * 4)
off_bnd = al(off_part + ((n + 4095) // 4096 + 2) * 4)
w = ws.cpu().numpy().view(np.uint32)
r = 65536 if n == 1 << 18 else None
S, M = 128, 28
ng = (n + 4 * r - 1) // (4 * r); spg = 4 * r // S; bpg = (spg + M - 1) // M
bnd = w[off_bnd // 4: off_bnd // 4 + ng * bpg * 4].reshape(-1, 4)
print("ws bytes", ws.numel(), "off_bnd", off_bnd, "bpg", bpg)
tmp = w[: n]  # pass input (tmp) after the pairwise pass -> the four-way pass read it
exp_in = np.concatenate([np.sort(t.cpu().numpy().view(np.uint32)[i:i + 2 * 32768]) for i in range(0, n, 2 * 32768)])
print("four-way input == runs of 65536 sorted:", np.array_equal(tmp, exp_in))
for b in range(16, 22):
    print(b, bnd[b].tolist(), sum(bnd[b].tolist()))
bw = ng * bpg * 4 + ((ng * spg + 3) & ~3)
off_samp0 = al(off_bnd + bw * 4)
samp0 = w[off_samp0 // 4: off_samp0 // 4 + n // 128]
print("off_samp0", off_samp0, "samples == input[::128]:", np.array_equal(samp0, tmp[::128]))
badS = np.nonzero(samp0 != tmp[::128])[0]
print("sample mismatches", badS.size, badS[:10], samp0[badS[:5]] if badS.size else "", tmp[::128][badS[:5]] if badS.size else "")
got = o.cpu().numpy().view(np.uint32)
exp = np.sort(t.cpu().numpy().view(np.uint32))
bad = np.nonzero(got != exp)[0]
print("wrong", bad.size, "first", bad[:5])
