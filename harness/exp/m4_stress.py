"""Randomized check of the merge sort's four-way passes (keys and key/value) against numpy:
random sizes from 2^15 to 2^23, adversarial key shapes (few distinct values, one outlier,
sorted / reversed runs, keys equal across runs, int32 negatives).  Prints one line per
failure and a summary; exits 1 on any failure.  Usage: python harness/exp/m4_stress.py [cases]"""
import importlib, os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
import torch
ls = importlib.import_module("radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd")
rng = np.random.default_rng(int(os.environ.get("SEED", "29")))
cases = int(sys.argv[1]) if len(sys.argv) > 1 else 120


def keys(n, shape):
    if shape == "uniform":
        return rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    if shape == "few":
        return rng.integers(0, int(rng.integers(1, 6)), n).astype(np.uint32) * np.uint32(0x9E3779B9)
    if shape == "outlier":
        a = np.full(n, 7, dtype=np.uint32)
        a[rng.integers(0, n, 3)] = rng.integers(0, 2**32, 3, dtype=np.uint64).astype(np.uint32)
        return a
    if shape == "runs":  # ascending / descending stretches of random length
        a = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        i = 0
        while i < n:
            L = int(rng.integers(1, 70000))
            seg = np.sort(a[i:i + L])
            a[i:i + L] = seg if rng.random() < 0.5 else seg[::-1]
            i += L
        return a
    if shape == "extremes":
        return rng.choice(np.array([0, 1, 0x7FFFFFFF, 0x80000000, 0xFFFFFFFE, 0xFFFFFFFF], dtype=np.uint32), n)
    raise ValueError(shape)


bad = 0
shapes = ["uniform", "few", "outlier", "runs", "extremes"]
for c in range(cases):
    n = int(2 ** rng.uniform(15, 23)) + int(rng.integers(0, 3))
    shape = shapes[c % len(shapes)]
    key = "i32" if rng.random() < 0.5 else "u32"
    a = keys(n, shape)
    vt = np.int32 if key == "i32" else np.uint32
    t = torch.from_numpy(a.view(np.int32).copy()).cuda()
    o = torch.empty_like(t)
    ls.sort_device(t, o, n, key=key, algo="merge")
    torch.cuda.synchronize()
    exp = np.sort(a.view(vt), kind="stable")
    got = o.cpu().numpy().view(vt)
    ok = np.array_equal(got, exp)
    if ok and c % 3 == 0:  # key/value: payload = input index, stable order
        v = torch.arange(n, dtype=torch.int32, device="cuda")
        ko, vo = torch.empty_like(t), torch.empty_like(t)
        ls.sort_pairs_device(t, v, ko, vo, n, key=key, algo="merge")
        torch.cuda.synchronize()
        perm = np.argsort(a.view(vt), kind="stable")
        ok = np.array_equal(ko.cpu().numpy().view(vt), exp) and np.array_equal(vo.cpu().numpy(), perm.astype(np.int32))
        kind = "pairs"
    else:
        kind = "keys"
    if not ok:
        bad += 1
        print(f"FAIL case {c}: n={n} shape={shape} key={key} ({kind})", flush=True)
print(f"{cases - bad}/{cases} ok", flush=True)
sys.exit(1 if bad else 0)
