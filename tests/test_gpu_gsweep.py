"""Both LSD radix implementations behind LABSORT_ALGO_RADIX, each forced with
LABSORT_RADIX_IMPL, against std::sort (the oracle):

  gather    gsweep.hip -- passes gather their tile run by run, sort it in LDS and write
            it contiguously; per-pass run tables; a final gathered copy (the default
            for 2^16 <= n < 2^25)
  onesweep  kernels.hip k_onesweep_p -- decoupled look-back scatter passes (the
            default outside that window)

Sizes straddle the 8192-key gather tile, the 32768-key tile-sort small path and the
64-tile scan groups; distributions cover trivial (skipped) passes, repeated keys and
digit columns that are empty or hold one key per tile (the gather's per-lane search
path)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED9000
GT = 8192  # gsweep tile (common.h GS_TILE)


def to_dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a).view(np.int32).copy()).cuda()


def from_dev(t):
    return t.cpu().numpy().view(np.uint32)


def ref(oracle, a, key):
    return oracle.sort_i32(a.view(np.int32)).view(np.uint32) if key == "i32" else oracle.sort_u32(a)


def sort_impl(ls, torch, a, key, impl, monkeypatch, inplace=False):
    monkeypatch.setenv("LABSORT_RADIX_IMPL", impl)
    n = a.size
    t = to_dev(torch, a)
    o = t if inplace else torch.empty_like(t)
    ws = torch.empty(max(ls.workspace_bytes(n, "radix"), 256), dtype=torch.uint8, device="cuda")
    ls.sort_device(t, o, n, key=key, algo="radix", workspace=ws)
    ls.workspace_status(ws, n, "radix")
    return from_dev(o)


SIZES = [1, 100, GT - 1, GT, GT + 1, 32769, 64 * GT + 1, 100_003, 262_145, (1 << 21) + 777, (1 << 22) + 12_345]


@pytest.mark.parametrize("impl", ["gather", "onesweep"])
@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("key", ["u32", "i32"])
def test_radix_impl_uniform(ls, oracle, torch_gpu, monkeypatch, impl, n, key):
    a = oracle.gen(n, SEED + n, "u32")
    np.testing.assert_array_equal(sort_impl(ls, torch_gpu, a, key, impl, monkeypatch), ref(oracle, a, key))


@pytest.mark.parametrize("impl", ["gather", "onesweep"])
@pytest.mark.parametrize("dist", ["u31", "mod100", "mod1000", "const", "sorted", "reversed", "lowbits"])
@pytest.mark.parametrize("inplace", [False, True])
def test_radix_impl_distributions(ls, oracle, torch_gpu, monkeypatch, impl, dist, inplace):
    n = 3 * (1 << 20) + 4321
    a = oracle.gen(n, SEED + 7, dist, param=12 if dist == "lowbits" else 0)
    np.testing.assert_array_equal(sort_impl(ls, torch_gpu, a, "u32", impl, monkeypatch, inplace), oracle.sort_u32(a))


def _sparse_cases(oracle, n):
    rng = np.random.default_rng(5)
    base = oracle.gen(n, SEED + 11, "u32")
    cases = {
        # 99 % zeros: 255 digit columns hold a key in only some tiles (runs of 0 or 1 keys)
        "mostly_zero": np.where(rng.random(n) < 0.99, 0, base).astype(np.uint32),
        # two values: digit columns 1..254 empty in every pass
        "two_values": np.where(base & 1, 0xFFFFFFFF, 0).astype(np.uint32),
        # even digit values only: every other digit column empty
        "even_digits": (base & np.uint32(0xFEFEFEFE)).astype(np.uint32),
        # one rare digit per byte position: columns of single keys
        "rare": np.where(rng.random(n) < 0.999, 0x80808080, base).astype(np.uint32),
    }
    return cases


@pytest.mark.parametrize("impl", ["gather", "onesweep"])
@pytest.mark.parametrize("case", ["mostly_zero", "two_values", "even_digits", "rare"])
@pytest.mark.parametrize("key", ["u32", "i32"])
def test_radix_impl_sparse_digits(ls, oracle, torch_gpu, monkeypatch, impl, case, key):
    n = (1 << 21) + 99
    a = _sparse_cases(oracle, n)[case]
    np.testing.assert_array_equal(sort_impl(ls, torch_gpu, a, key, impl, monkeypatch), ref(oracle, a, key))


@pytest.mark.parametrize("mask", [0xFFFF00FF, 0x0F0F0F0F, 0xFF0000FF, 0x000000FF, 0x80000001, 0xFF000000])
def test_gather_pass_structure(ls, oracle, torch_gpu, monkeypatch, mask):
    """trivial passes skipped on the device: the run tables of the last active pass feed
    the next active one and the final copy"""
    n = (1 << 20) + 333
    a = oracle.gen(n, SEED + 21, "u32") & np.uint32(mask)
    for key in ("u32", "i32"):
        np.testing.assert_array_equal(sort_impl(ls, torch_gpu, a, key, "gather", monkeypatch), ref(oracle, a, key))


def test_gather_default_window(ls):
    """which implementation LABSORT_ALGO_RADIX runs, as api.hip decides"""
    assert ls.radix_impl(1 << 15) == "onesweep" and ls.radix_impl(1 << 16) == "gather"
    assert ls.radix_impl((1 << 25) - 1) == "gather" and ls.radix_impl(1 << 25) == "onesweep"


# ---- the fused small path (gsweep.hip, at most 128 tiles = 2^20 keys): no scan launches;
# each pass derives its tile's runs from the previous pass's rows and accumulated digit
# totals (no memset: pass 1 reads pass 0's rows)
@pytest.mark.parametrize("mask", [0xFFFF00FF, 0x0F0F0F0F, 0xFF0000FF, 0x000000FF, 0x80000001, 0xFF000000, 0x00FFFF00])
def test_gather_fused_pass_structure(ls, oracle, torch_gpu, monkeypatch, mask):
    """skipped passes forward the digit totals they received (acc[p] <- acc[p - 1])"""
    n = (1 << 20) - 333
    a = oracle.gen(n, SEED + 31, "u32") & np.uint32(mask)
    for key in ("u32", "i32"):
        np.testing.assert_array_equal(sort_impl(ls, torch_gpu, a, key, "gather", monkeypatch), ref(oracle, a, key))


@pytest.mark.parametrize("dist", ["u31", "mod100", "mod1000", "const", "sorted", "reversed", "lowbits"])
@pytest.mark.parametrize("n", [GT + 3, 1 << 20])
def test_gather_fused_distributions(ls, oracle, torch_gpu, monkeypatch, dist, n):
    a = oracle.gen(n, SEED + 33, dist, param=12 if dist == "lowbits" else 0)
    np.testing.assert_array_equal(sort_impl(ls, torch_gpu, a, "u32", "gather", monkeypatch, inplace=(n & 1) == 1),
                                  oracle.sort_u32(a))


@pytest.mark.parametrize("case", ["mostly_zero", "two_values", "even_digits", "rare"])
def test_gather_fused_sparse_digits(ls, oracle, torch_gpu, monkeypatch, case):
    """tiles that meet many digits (more than one chunk of runs in the prologue)"""
    a = _sparse_cases(oracle, (1 << 20) - 5)[case]
    for key in ("u32", "i32"):
        np.testing.assert_array_equal(sort_impl(ls, torch_gpu, a, key, "gather", monkeypatch), ref(oracle, a, key))


def test_gather_fused_repeat_same_workspace(ls, oracle, torch_gpu, monkeypatch):
    """back-to-back sorts on one workspace: the accumulators a sort leaves behind (and
    garbage before the first) never leak into the next sort"""
    monkeypatch.setenv("LABSORT_RADIX_IMPL", "gather")
    n = 500_000
    ws = torch_gpu.full((max(ls.workspace_bytes(n, "radix"), 256),), 0xA5, dtype=torch_gpu.uint8, device="cuda")
    for i, dist in enumerate(["u32", "mod1000", "u32", "lowbits", "sorted"]):
        a = oracle.gen(n, SEED + 40 + i, dist, param=12 if dist == "lowbits" else 0)
        t = to_dev(torch_gpu, a)
        o = torch_gpu.empty_like(t)
        ls.sort_device(t, o, n, key="u32", algo="radix", workspace=ws)
        ls.workspace_status(ws, n, "radix")
        np.testing.assert_array_equal(from_dev(o), oracle.sort_u32(a))


@pytest.mark.parametrize("inplace", [False, True])
def test_onesweep_lookback_clear(ls, oracle, torch_gpu, monkeypatch, inplace):
    """the look-back clear folded into a launch; a dirty workspace from the previous sort
    must not leak"""
    n = (1 << 22) + 4097
    for i in range(2):
        a = oracle.gen(n, SEED + 50 + i, "u32")
        np.testing.assert_array_equal(sort_impl(ls, torch_gpu, a, "u32", "onesweep", monkeypatch, inplace),
                                      oracle.sort_u32(a))
