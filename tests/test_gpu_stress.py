"""Randomized parity across every sort entry point (the seeded short form of
harness/exp/sort_stress.py): device radix at the size's default implementation and forced
onesweep / gathered passes, merge, AUTO, stable key/value radix and merge, host-pointer
radix and merge; log-uniform sizes to 2^22 and edge sizes, in place or not, u32 / i32
order, adversarial key shapes.  Expected results from numpy's stable sort (integer keys:
any correct sort is bit-exact to it)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SHAPES = ["uniform", "u31", "few", "byte", "sorted", "reversed", "const", "extremes", "runs"]
MODES = ["radix", "radix:onesweep", "radix:gather", "merge", "auto", "pairs:radix", "pairs:merge", "host:radix",
         "host:merge"]


def _keys(rng, n, shape):
    if shape == "uniform":
        return rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    if shape == "u31":
        return rng.integers(0, 2**31, n, dtype=np.uint64).astype(np.uint32)
    if shape == "few":
        return rng.integers(0, int(rng.integers(1, 9)), n).astype(np.uint32) * np.uint32(0x9E3779B9)
    if shape == "byte":
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
    a = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)  # "runs"
    i = 0
    while i < n:
        L = int(rng.integers(1, 70000))
        seg = np.sort(a[i:i + L])
        a[i:i + L] = seg if rng.random() < 0.5 else seg[::-1]
        i += L
    return a


@pytest.mark.parametrize("seed", [61, 62, 63])
def test_randomized_entry_points(ls, torch_gpu, monkeypatch, seed):
    torch = torch_gpu
    rng = np.random.default_rng(seed)
    tile, mtile = ls.tile_keys(), ls.merge_tile_keys()
    edge = [0, 1, 2, 63, 64, 65, 4095, 4096, 4097, 16384, 16385, tile - 1, tile, tile + 1, mtile - 1, mtile + 1,
            3 * mtile + 127, (1 << 16) + 1, (1 << 20) - 1, (1 << 20) + 1]
    failures = []
    for c in range(120):
        n = edge[c % len(edge)] if c % 3 == 0 else int(2 ** rng.uniform(0, 22))
        shape = SHAPES[int(rng.integers(0, len(SHAPES)))]
        mode = MODES[c % len(MODES)]
        key = "i32" if rng.random() < 0.5 else "u32"
        inplace = rng.random() < 0.3
        kind, _, impl = mode.partition(":")
        a = _keys(rng, n, shape)
        vt = np.int32 if key == "i32" else np.uint32
        exp = np.sort(a.view(vt), kind="stable")
        if impl and kind == "radix":
            monkeypatch.setenv("LABSORT_RADIX_IMPL", impl)
        else:
            monkeypatch.delenv("LABSORT_RADIX_IMPL", raising=False)
        if kind in ("radix", "merge", "auto"):
            t = torch.from_numpy(a.view(np.int32).copy()).cuda()
            o = t if inplace else torch.empty_like(t)
            ls.sort_device(t, o, n, key=key, algo=kind)
            torch.cuda.synchronize()
            ok = np.array_equal(o.cpu().numpy().view(vt), exp)
            if ok and not inplace:
                ok = np.array_equal(t.cpu().numpy().view(np.uint32), a)
        elif kind == "pairs":
            t = torch.from_numpy(a.view(np.int32).copy()).cuda()
            v = torch.arange(n, dtype=torch.int32, device="cuda")
            ko, vo = (t, v) if inplace else (torch.empty_like(t), torch.empty_like(v))
            ls.sort_pairs_device(t, v, ko, vo, n, key=key, algo=impl)
            torch.cuda.synchronize()
            perm = np.argsort(a.view(vt), kind="stable").astype(np.int32)
            ok = np.array_equal(ko.cpu().numpy().view(vt), exp) and np.array_equal(vo.cpu().numpy(), perm)
        else:
            h = a.view(vt).copy()
            ls.sort_host(h, algo=impl)
            ok = np.array_equal(h, exp)
        if not ok:
            failures.append(f"case {c}: {mode} n={n} {shape} {key} inplace={inplace}")
    assert not failures, failures
