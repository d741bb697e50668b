"""A/B of the 2^28 key/value (MODE=pairs, default) or keys-only (MODE=keys) radix sort across liblabsort builds (paths on the command
line, relative to the repo root), alternating, each sort event-timed on the stream, plus
the per-launch onesweep time from the library's own timing class.  Only C-ABI entry points
every round's build exports are used (labsort_fill, labsort_sort_pairs_device, timing).
Usage: python harness/exp/pairs_ab.py LIB_A LIB_B [reps]"""
import ctypes, json, os, sys
import torch

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
libs = [a for a in sys.argv[1:] if not a.isdigit()]
reps = int(next((a for a in sys.argv[1:] if a.isdigit()), "3"))
n = 1 << int(os.environ.get("LOG2N", "28"))
p, sz = ctypes.c_void_p, ctypes.c_size_t
L = {}
for lib in libs:
    h = ctypes.CDLL(os.path.join(R, lib))
    h.labsort_fill.argtypes = [p, sz, ctypes.c_uint64, ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, p]
    h.labsort_pairs_workspace_bytes.argtypes = [sz, ctypes.c_int]
    h.labsort_pairs_workspace_bytes.restype = sz
    h.labsort_sort_pairs_device.argtypes = [p, p, p, p, sz, ctypes.c_int, ctypes.c_int, p, sz, p]
    h.labsort_workspace_bytes.argtypes = [sz, ctypes.c_int]
    h.labsort_workspace_bytes.restype = sz
    h.labsort_sort_device.argtypes = [p, p, sz, ctypes.c_int, ctypes.c_int, p, sz, p]
    h.labsort_timing_read.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong)]
    L[lib] = h
k = torch.empty(n, dtype=torch.int32, device="cuda")
v = torch.arange(n, dtype=torch.int32, device="cuda")
ko, vo = torch.empty_like(k), torch.empty_like(v)
st = torch.cuda.current_stream().cuda_stream
first = L[libs[0]]
assert first.labsort_fill(k.data_ptr(), n, 0x5EED0003, 0, 0, 0, p(st)) == 0
mode = os.environ.get("MODE", "pairs")  # pairs | keys | merge | pairsmerge (key/value merge sort)
keys = mode in ("keys", "merge")
algo = 1 if mode in ("merge", "pairsmerge") else 0
wsb = max((h.labsort_workspace_bytes(n, algo) if keys else h.labsort_pairs_workspace_bytes(n, algo)) for h in L.values())
ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
ref = None
for r in range(reps):
    for lib, h in L.items():
        if keys:
            call = lambda: h.labsort_sort_device(k.data_ptr(), ko.data_ptr(), n, 0, algo, ws.data_ptr(), wsb, p(st))
        else:
            call = lambda: h.labsort_sort_pairs_device(k.data_ptr(), v.data_ptr(), ko.data_ptr(), vo.data_ptr(), n, 0, algo,
                                                       ws.data_ptr(), wsb, p(st))
        for _ in range(3):
            assert call() == 0
        torch.cuda.synchronize()
        h.labsort_timing_enable(1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            assert call() == 0
        e1.record()
        torch.cuda.synchronize()
        cls = {}
        for name, c in (("onesweep", 1), ("tile_sort", 2), ("merge", 3), ("merge4", 8)):
            ms, cnt = ctypes.c_double(0.0), ctypes.c_longlong(0)
            if h.labsort_timing_read(c, ctypes.byref(ms), ctypes.byref(cnt)) == 0 and cnt.value:
                cls[name] = (round(ms.value / cnt.value, 4), cnt.value // 10)
        h.labsort_timing_enable(0)
        sig = (int(ko[:: 1 << 12].sum().item()), int(vo[:: 1 << 12].sum().item()))
        ref = ref or sig
        print(json.dumps({"mode": mode, "lib": lib, "rep": r, "sort_ms": round(e0.elapsed_time(e1) / 10, 4),
                          "per_launch_ms_and_launches_per_sort": cls, "same_output": sig == ref}), flush=True)
