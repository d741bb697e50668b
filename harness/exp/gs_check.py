"""Gathered radix (gsweep.hip) vs the onesweep passes on the same device input:
bit-exact equality and per-sort time, for a few sizes and distributions."""
import importlib, os, sys, time
import torch
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
ls = importlib.import_module("radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd")


def run(n, dist, key, impl, reps=5, param=None, algo="radix"):
    os.environ["LABSORT_RADIX_IMPL"] = impl
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    ls.fill(t, n, 0x5EED0003, dist, param=param if param is not None else (5 if dist == "lowbits" else 0))
    o = torch.empty_like(t)
    ws = torch.empty(ls.workspace_bytes(n, algo), dtype=torch.uint8, device="cuda")
    ls.sort_device(t, o, n, key=key, algo=algo, workspace=ws)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a = time.perf_counter()
        ls.sort_device(t, o, n, key=key, algo=algo, workspace=ws)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - a)
    ls.workspace_status(ws, n, algo)
    return o, sorted(ts)[len(ts) // 2] * 1e3


if len(sys.argv) > 1 and sys.argv[1] == "small":
    for lg in range(14, 23):
        n = 1 << lg
        _, tg = run(n, "u32", "u32", "gather", reps=15)
        _, to = run(n, "u32", "u32", "onesweep", reps=15)
        os.environ["LABSORT_RADIX_IMPL"] = ""
        t = torch.empty(n, dtype=torch.int32, device="cuda"); ls.fill(t, n, 3, "u32"); o = torch.empty_like(t)
        ws = torch.empty(ls.workspace_bytes(n, "merge"), dtype=torch.uint8, device="cuda")
        ts = []
        for _ in range(15):
            a = time.perf_counter(); ls.sort_device(t, o, n, algo="merge", workspace=ws); torch.cuda.synchronize()
            ts.append(time.perf_counter() - a)
        print(f"2^{lg} gather {tg:.3f} onesweep {to:.3f} merge {sorted(ts)[7]*1e3:.3f} ms", flush=True)
    sys.exit(0)
if len(sys.argv) > 1 and sys.argv[1] == "sizes":
    for lg in range(22, 29):
        for dist in ("u32", "mod1000", "u31"):
            _, tg = run(1 << lg, dist, "u32", "gather", reps=9)
            _, to = run(1 << lg, dist, "u32", "onesweep", reps=9)
            print(f"2^{lg} {dist:8s} gather {tg:.3f} ms  onesweep {to:.3f} ms  ratio {to / tg:.2f}", flush=True)
    sys.exit(0)
if len(sys.argv) > 1 and sys.argv[1] == "lowbits":  # few distinct digit values
    for p in (1, 2, 4, 9, 12, 17):
        _, tg = run(1 << 28, "lowbits", "u32", "gather", reps=5, param=p)
        _, to = run(1 << 28, "lowbits", "u32", "onesweep", reps=5, param=p)
        _, tm = run(1 << 28, "lowbits", "u32", "", reps=3, param=p, algo="merge")
        print(f"2^28 lowbits {p:2d}: gather {tg:.3f} onesweep {to:.3f} merge {tm:.3f} ms", flush=True)
    sys.exit(0)
if len(sys.argv) > 1 and sys.argv[1] == "dists":  # every generator distribution at 2^28
    for d in ("u32", "u31", "mod100", "mod1000", "sorted", "reversed", "const"):
        p = (1 << 28) if d == "reversed" else (77 if d == "const" else None)
        _, to = run(1 << 28, d, "u32", "onesweep", reps=5, param=p)
        _, tg = run(1 << 28, d, "u32", "gather", reps=5, param=p)
        _, tm = run(1 << 28, d, "u32", "", reps=3, param=p, algo="merge")
        print(f"2^28 {d:8s}: onesweep {to:.3f} gather {tg:.3f} merge {tm:.3f} ms", flush=True)
    sys.exit(0)
if len(sys.argv) > 1 and sys.argv[1] == "time":
    _, tg = run(1 << 28, "u32", "u32", "gather", reps=15)
    _, to = run(1 << 28, "u32", "u32", "onesweep", reps=15)
    print(f"{os.path.basename(os.environ.get('LABSORT_LIBRARY', 'default'))}: gather {tg:.3f} ms  onesweep {to:.3f} ms")
    sys.exit(0)
if len(sys.argv) > 1 and sys.argv[1] == "prof":
    run(1 << int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 28, sys.argv[3] if len(sys.argv) > 3 else "u32", "u32",
        sys.argv[4] if len(sys.argv) > 4 else "gather", reps=10)
    sys.exit(0)
for n, dist, key in [(1 << 22, "u32", "u32"), ((1 << 22) + 12345, "mod100", "i32"), ((1 << 24) + 7, "u32", "i32"),
                     (1 << 24, "const", "u32"), (1 << 24, "lowbits", "u32"), (1 << 28, "u32", "u32")]:
    a, ta = run(n, dist, key, "gather")
    b, tb = run(n, dist, key, "onesweep")
    same = torch.equal(a, b)
    print(f"n={n} {dist} {key}: gather {ta:.3f} ms, onesweep {tb:.3f} ms, equal={same}", flush=True)
    if not same:
        bad = (a != b).nonzero()
        print("  first mismatch at", int(bad[0]), "count", bad.numel())
        sys.exit(1)
