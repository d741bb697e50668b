"""labsort_sort_host (order_array's path) with and without the host pipeline
(LABSORT_HOST_PIPE), pageable int32 host arrays, median of 3, verified."""
import importlib, json, os, sys, time
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
import numpy as np
import torch
ls = importlib.import_module("radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd")
for lg in [int(x) for x in os.environ.get("LOG2NS", "24 26 28 30").split()]:
    n = 1 << lg
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    ls.fill(t, n, 0x5EED0005, "u31")
    src = t.cpu().numpy(); del t; torch.cuda.empty_cache()
    exp = None
    row = {"n": n}
    for pipe in ("1", "0"):
        os.environ["LABSORT_HOST_PIPE"] = pipe
        w = src.copy(); ls.sort_host(w, algo="auto")
        if exp is None:
            exp = w.copy(); assert bool((exp[1:] >= exp[:-1]).all())
        assert np.array_equal(w, exp)
        ts = []
        for _ in range(3):
            np.copyto(w, src); a = time.perf_counter(); ls.sort_host(w, algo="auto"); ts.append(time.perf_counter() - a)
        assert np.array_equal(w, exp)
        row["pipe" if pipe == "1" else "plain"] = round(sorted(ts)[1] * 1e3, 2)
    print(json.dumps(row), flush=True)
