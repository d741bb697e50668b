"""k_tile_sort (one-shot) vs k_tile_sort_p (persistent, pipelined): merge sort of 2^28
keys, per-kernel times via the timing hooks, and bit-exact equality."""
import importlib, os, sys, subprocess
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if len(sys.argv) == 1:
    for p in ("0", "1"):
        subprocess.run([sys.executable, __file__, p], env=dict(os.environ, LABSORT_TS_PERSIST=p), check=True)
    sys.exit(0)
import torch, time, hashlib
sys.path.insert(0, R)
ls = importlib.import_module("radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd")
n = 1 << 28
t = torch.empty(n, dtype=torch.int32, device="cuda"); ls.fill(t, n, 0x5EED0003, "u32"); o = torch.empty_like(t)
ws = torch.empty(ls.workspace_bytes(n, "merge"), dtype=torch.uint8, device="cuda")
ls.sort_device(t, o, n, algo="merge", workspace=ws); torch.cuda.synchronize()
ls.timing_enable(True)
a = time.perf_counter()
for _ in range(10):
    ls.sort_device(t, o, n, algo="merge", workspace=ws)
torch.cuda.synchronize()
el = (time.perf_counter() - a) / 10 * 1e3
ts, tc = ls.timing_read("tile_sort"); ms, mc = ls.timing_read("merge")
ls.timing_enable(False)
h = hashlib.sha256(o.cpu().numpy().tobytes()).hexdigest()[:16]
print(f"persist={sys.argv[1]}: merge sort {el:.3f} ms, tile sort {ts / tc:.4f} ms, merge pass {ms / mc:.4f} ms, sha {h}")
