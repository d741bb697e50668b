"""Diagnostic: the host-pointer path (order_array / labsort_sort_host) end to end.

For n = 2^8 .. 2^28 uniform int32 keys in [0, 2^31): median wall time of
labsort_sort_host (H2D + device sort + D2H + sync), next to the device-only sort
and plain pageable / pinned copies of the same bytes through torch.
Prints one JSON line per n."""
import ctypes, importlib, json, os, sys, time
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
import numpy as np
import torch
ls = importlib.import_module("radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd")


def med(f, reps):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2] * 1e3


rng = np.random.default_rng(1)
for lg in [int(x) for x in os.environ.get("LOGS", "8 12 16 20 24 28").split()]:
    n = 1 << lg
    reps = 20 if lg <= 20 else 5
    base = rng.integers(0, 1 << 31, n, dtype=np.int32)
    a = base.copy()
    ls.order_array(a)  # warm-up (allocates the cached device buffers)
    assert np.array_equal(a, np.sort(base))

    def host_sort():
        a[:] = base
        ls.order_array(a)
    t_copy_only = med(lambda: a.__setitem__(slice(None), base), reps)
    t_host = med(host_sort, reps) - t_copy_only
    d = torch.from_numpy(base).cuda()
    o = torch.empty_like(d)
    ws = torch.empty(ls.workspace_bytes(n), dtype=torch.uint8, device="cuda")

    def dev_sort():
        ls.sort_device(d, o, n, key="i32", workspace=ws)
        torch.cuda.synchronize()
    t_dev = med(dev_sort, reps)
    pg = torch.from_numpy(base)
    pin = pg.pin_memory()
    t_h2d_pageable = med(lambda: (d.copy_(pg), torch.cuda.synchronize()), reps)
    t_h2d_pinned = med(lambda: (d.copy_(pin, non_blocking=True), torch.cuda.synchronize()), reps)
    t_d2h_pageable = med(lambda: (pg.copy_(d), torch.cuda.synchronize()), reps)
    t_d2h_pinned = med(lambda: (pin.copy_(d, non_blocking=True), torch.cuda.synchronize()), reps)
    print(json.dumps({"log2n": lg, "order_array_ms": round(t_host, 4), "device_sort_ms": round(t_dev, 4),
                      "h2d_pageable_ms": round(t_h2d_pageable, 4), "h2d_pinned_ms": round(t_h2d_pinned, 4),
                      "d2h_pageable_ms": round(t_d2h_pageable, 4), "d2h_pinned_ms": round(t_d2h_pinned, 4),
                      "GBps_h2d_pinned": round(4 * n / t_h2d_pinned / 1e6, 1)}), flush=True)
