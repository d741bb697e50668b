"""Diagnostic: device-resident sort time (median of HIP-event-timed calls) for radix
and merge at small n, to place the size crossover of LABSORT_ALGO_AUTO."""
import importlib, json, os, sys
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
import torch
ls = importlib.import_module("radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd")
# warm the clocks first: without this the first sizes read ~0.13 ms for one small launch
_w = torch.empty(1 << 22, dtype=torch.int32, device="cuda")
ls.fill(_w, _w.numel(), 1, "u32")
for _ in range(200):
    ls.sort_device(_w, _w, _w.numel(), algo="merge")
torch.cuda.synchronize()
for n in [int(x) for x in os.environ.get("NS", "").split()] or [256, 4096, 32768, 32769, 49152, 65536, 98304, 131072, 196608, 262144, 524288, 1 << 20, 1 << 21, 1 << 22, 1 << 23]:
    d = torch.empty(n, dtype=torch.int32, device="cuda")
    ls.fill(d, n, 0x5EED0002, os.environ.get("DIST", "u32"), param=int(os.environ.get("PARAM", "0")))
    o = torch.empty_like(d)
    row = {"n": n}
    ref = torch.sort(d.to(torch.int64) & 0xFFFFFFFF)[0].to(torch.int32)
    for name in os.environ.get("IMPLS", "radix merge").split():
        # radix:<impl> selects LABSORT_RADIX_IMPL (small | gather | onesweep)
        algo, _, impl = name.partition(":")
        if impl:
            os.environ["LABSORT_RADIX_IMPL"] = impl
        else:
            os.environ.pop("LABSORT_RADIX_IMPL", None)
        ws = torch.empty(max(ls.workspace_bytes(n, algo), 256), dtype=torch.uint8, device="cuda")
        for _ in range(3):
            ls.sort_device(d, o, n, algo=algo, workspace=ws)
        ts = []
        for _ in range(25):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            ls.sort_device(d, o, n, algo=algo, workspace=ws)
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        ts.sort()
        ls.workspace_status(ws, n, algo)
        assert torch.equal(o, ref), (n, name)
        row[name + "_ms"] = round(ts[len(ts) // 2], 4)
        if os.environ.get("B2B"):  # also 50 sorts back to back (bench.py's config-2 timing)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(50):
                ls.sort_device(d, o, n, algo=algo, workspace=ws)
            b.record()
            b.synchronize()
            row[name + "_b2b_ms"] = round(a.elapsed_time(b) / 50, 4)
    print(json.dumps(row), flush=True)
