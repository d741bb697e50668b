"""Key/value sort (labsort_sort_pairs_device) per size: radix and merge, median of 9."""
import importlib, os, sys, time
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
import torch
ls = importlib.import_module("radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd")
for lg in [int(x) for x in os.environ.get("LOG2NS", "16 18 20 22 24 26 28").split()]:
    n = 1 << lg
    k = torch.empty(n, dtype=torch.int32, device="cuda"); ls.fill(k, n, 0x5EED0011, os.environ.get("DIST", "u32"), param=int(os.environ.get("PARAM", "0")))
    v = torch.arange(n, dtype=torch.int32, device="cuda")
    ko, vo = torch.empty_like(k), torch.empty_like(v)
    row = [f"2^{lg}"]
    for algo in ("radix", "merge"):
        ws = torch.empty(max(ls.pairs_workspace_bytes(n, algo), 256), dtype=torch.uint8, device="cuda")
        ls.sort_pairs_device(k, v, ko, vo, n, algo=algo, workspace=ws); torch.cuda.synchronize()
        ts = []
        for _ in range(9):
            a = time.perf_counter(); ls.sort_pairs_device(k, v, ko, vo, n, algo=algo, workspace=ws)
            torch.cuda.synchronize(); ts.append(time.perf_counter() - a)
        row.append(f"{algo} {sorted(ts)[4]*1e3:.3f} ms")
        del ws
    print("  ".join(row), flush=True)
