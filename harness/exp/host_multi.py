"""The one-process multi-GPU host sort (labsort_sort_host_ranks) on ONE GPU with p ranks
sharing it (peer-copy exchange), n = 2^28 int32 keys from a host buffer: per-phase
times (labsort_multi_timing) next to the single-GPU labsort_sort_host.  On one device
the ranks' H2D copies share one PCIe link, so this prices the schedule's overheads
(plan, exchange as D2D copies, merge), not the 8-link host path."""
import importlib, json, os, sys, time
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R); sys.path.insert(0, R + "/oracle")
import numpy as np
import torch  # noqa: F401  (one HIP runtime)
import oracle as O
ls = importlib.import_module("radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd")
n = 1 << int(os.environ.get("LOG2N", "28"))
src = O.gen(n, 0x5EED0005, "u32").view(np.int32)
exp = np.sort(src)
a = src.copy()
ls.sort_host(a, algo="radix")  # warm-up
ts = []
for _ in range(3):
    a = src.copy()
    t0 = time.perf_counter(); ls.sort_host(a, algo="radix"); ts.append((time.perf_counter() - t0) * 1e3)
assert np.array_equal(a, exp)
print(json.dumps({"n": n, "path": "labsort_sort_host (1 GPU)", "ms": round(sorted(ts)[1], 3)}), flush=True)
for p in (1, 2, 4, 8):
    a = src.copy()
    ls.sort_host_ranks(a, [0] * p, transport="peer")  # warm-up (buffers)
    rows = []
    for _ in range(3):
        a = src.copy()
        t0 = time.perf_counter(); ls.sort_host_ranks(a, [0] * p, transport="peer"); el = (time.perf_counter() - t0) * 1e3
        ph, sent = ls.multi_timing()
        rows.append((el, ph, sent))
    assert np.array_equal(a, exp), p
    el, ph, sent = sorted(rows, key=lambda r: r[0])[1]
    print(json.dumps({"n": n, "path": f"labsort_sort_host_ranks, {p} ranks on one GPU (peer copies)", "ms": round(el, 3),
                      "phases_ms": {k: round(v, 3) for k, v in ph.items()}, "max_sent_bytes": sent}), flush=True)
