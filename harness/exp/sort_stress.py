"""Randomized end-to-end check of every sort entry point against numpy: device sorts by
radix (each implementation: the size's default, LABSORT_RADIX_IMPL=onesweep / gather),
merge and AUTO; key/value sorts (stable: payload = input index); host-pointer
sorts (order_array's path, pipelined from 2^27 keys); with RANKS=1 also the multi-GPU
schedule with 2-8 ranks sharing one GPU (labsort_sort_host_ranks, peer copies).
Sizes log-uniform from 0 to 2^25 plus edge sizes (0, 1, powers of two +-1, tile and
sample multiples), in place or not, u32 / i32 order, adversarial key shapes.  One line
per failure and a summary; exit 1 on any failure.
Usage: python harness/exp/sort_stress.py [cases]   (SEED, MAXLOG env)"""
import importlib, os, sys, time
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
import torch
ls = importlib.import_module("radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd")
rng = np.random.default_rng(int(os.environ.get("SEED", "41")))
cases = int(sys.argv[1]) if len(sys.argv) > 1 else 300
maxlog = float(os.environ.get("MAXLOG", "25"))
TILE, MTILE = ls.tile_keys(), ls.merge_tile_keys()
EDGE = [0, 1, 2, 3, 63, 64, 65, 255, 256, 257, 4095, 4096, 4097, 8191, 8192, 8193, 16383, 16384, 16385,
        TILE - 1, TILE, TILE + 1, MTILE - 1, MTILE, MTILE + 1, 3 * MTILE + 127, (1 << 16), (1 << 16) + 1,
        (1 << 18) + 5, (1 << 20) - 1, (1 << 20), (1 << 20) + 1, (1 << 24) + 3, (1 << 25) - 1]


def keys(n, shape):
    if shape == "uniform":
        return rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    if shape == "u31":
        return rng.integers(0, 2**31, n, dtype=np.uint64).astype(np.uint32)
    if shape == "few":
        return (rng.integers(0, int(rng.integers(1, 9)), n).astype(np.uint32) * np.uint32(0x9E3779B9))
    if shape == "byte":  # one varying byte at a random position: three passes skipped
        b = int(rng.integers(0, 4))
        return (rng.integers(0, 256, n).astype(np.uint32) << np.uint32(8 * b)) | np.uint32(0x01010101 & ~(0xFF << (8 * b)))
    if shape == "sorted":
        return np.sort(rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32))
    if shape == "reversed":
        return np.sort(rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32))[::-1].copy()
    if shape == "const":
        return np.full(n, int(rng.integers(0, 2**32)), dtype=np.uint32)
    if shape == "extremes":
        return rng.choice(np.array([0, 1, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFE, 0xFFFFFFFF], dtype=np.uint32), n)
    if shape == "runs":
        a = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        i = 0
        while i < n:
            L = int(rng.integers(1, 70000))
            seg = np.sort(a[i:i + L])
            a[i:i + L] = seg if rng.random() < 0.5 else seg[::-1]
            i += L
        return a
    raise ValueError(shape)


SHAPES = ["uniform", "u31", "few", "byte", "sorted", "reversed", "const", "extremes", "runs"]
MODES = ["radix", "radix:onesweep", "radix:gather", "merge", "auto", "pairs:radix", "pairs:merge",
         "host:radix", "host:merge"] + (["ranks:peer"] if os.environ.get("RANKS") else [])
bad = 0
counts = {}
t0 = time.time()
for c in range(cases):
    n = EDGE[c % len(EDGE)] if c % 4 == 0 else int(2 ** rng.uniform(0, maxlog))
    shape = SHAPES[int(rng.integers(0, len(SHAPES)))]
    mode = MODES[c % len(MODES)]
    key = "i32" if rng.random() < 0.5 else "u32"
    inplace = rng.random() < 0.3
    kind, _, impl = mode.partition(":")
    a = keys(n, shape)
    vt = np.int32 if key == "i32" else np.uint32
    exp = np.sort(a.view(vt), kind="stable")
    if impl and kind == "radix":
        os.environ["LABSORT_RADIX_IMPL"] = impl
    else:
        os.environ.pop("LABSORT_RADIX_IMPL", None)
    ok = True
    try:
        if kind in ("radix", "merge", "auto"):
            t = torch.from_numpy(a.view(np.int32).copy()).cuda()
            o = t if inplace else torch.empty_like(t)
            ls.sort_device(t, o, n, key=key, algo=kind)
            torch.cuda.synchronize()
            ok = np.array_equal(o.cpu().numpy().view(vt), exp)
            if ok and not inplace:
                ok = np.array_equal(t.cpu().numpy().view(np.uint32), a)  # input untouched
        elif kind == "pairs":
            t = torch.from_numpy(a.view(np.int32).copy()).cuda()
            v = torch.arange(n, dtype=torch.int32, device="cuda")
            ko, vo = (t, v) if inplace else (torch.empty_like(t), torch.empty_like(v))
            ls.sort_pairs_device(t, v, ko, vo, n, key=key, algo=impl)
            torch.cuda.synchronize()
            perm = np.argsort(a.view(vt), kind="stable").astype(np.int32)
            ok = np.array_equal(ko.cpu().numpy().view(vt), exp) and np.array_equal(vo.cpu().numpy(), perm)
        elif kind == "ranks":  # the multi-GPU schedule with p ranks sharing this GPU (peer copies)
            p = int(rng.integers(2, 9))
            h = a.view(vt).copy()
            ls.sort_host_ranks(h, [0] * p, transport=impl)
            ok = np.array_equal(h, exp)
            mode = f"ranks:{impl}:p{p}"
        else:  # host pointer
            h = a.view(vt).copy()
            ls.sort_host(h, algo=impl)
            ok = np.array_equal(h, exp)
    except Exception as e:  # noqa: BLE001
        ok = False
        print(f"case {c}: {mode} n={n} {shape} {key} inplace={inplace}: EXCEPTION {e}", flush=True)
    counts[mode] = counts.get(mode, 0) + 1
    if not ok:
        bad += 1
        print(f"case {c}: {mode} n={n} {shape} {key} inplace={inplace}: MISMATCH", flush=True)
    if c % 100 == 99:
        print(f"... {c + 1} cases, {bad} failed, {time.time() - t0:.0f} s", flush=True)
os.environ.pop("LABSORT_RADIX_IMPL", None)
print(f"{cases - bad}/{cases} ok (seed {os.environ.get('SEED', '41')}, sizes to 2^{maxlog:g}); per mode {counts}")
sys.exit(1 if bad else 0)
