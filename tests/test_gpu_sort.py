"""GPU parity tests: every path through liblabsort.so's C-ABI against the oracle
(std::sort, the spec of order_array: letra.pdf p.3) on the same
seeded inputs.  Bit-exact equality is the bar (integer work)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED0000


def to_dev(torch, a):
    a = np.ascontiguousarray(a)
    return torch.from_numpy(a.view(np.int32).copy()).cuda()


def from_dev(t, dtype=np.uint32):
    return t.cpu().numpy().view(dtype)


def ref_sort(oracle, a, key):
    return oracle.sort_i32(a.view(np.int32)).view(np.uint32) if key == "i32" else oracle.sort_u32(a)


# ---- generator ------------------------------------------------------------------------
@pytest.mark.parametrize("dist", ["u32", "u31", "mod100", "mod1000", "sorted", "reversed", "const", "lowbits"])
def test_fill_matches_oracle_generator(ls, oracle, torch_gpu, dist):
    torch = torch_gpu
    n, first = 100_003, 12_345
    param = 77 if dist in ("const",) else (13 if dist == "lowbits" else 0)
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    ls.fill(t, n, SEED + 1, dist, param=param, first=first)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(from_dev(t), oracle.gen(n, SEED + 1, dist, param=param, first=first))


# ---- radix_sort_kernel's job: 64-key tiles by bit splits ---------------------------------
@pytest.mark.parametrize("key", ["u32", "i32"])
@pytest.mark.parametrize("dist", ["u32", "mod100", "sorted", "reversed"])
def test_wave_tile_sort(ls, oracle, torch_gpu, key, dist):
    torch = torch_gpu
    n = (1 << 16) + 37
    a = oracle.gen(n, SEED + 2, dist)
    t = to_dev(torch, a)
    ls.wave_tile_sort(t, n, key=key)
    torch.cuda.synchronize()
    got = from_dev(t)
    for s in range(0, n, 64):
        np.testing.assert_array_equal(got[s:s + 64], ref_sort(oracle, a[s:s + 64].copy(), key))


# ---- LDS tile sort (stage 1+2 counterpart) ---------------------------------------------
@pytest.mark.parametrize("key", ["u32", "i32"])
@pytest.mark.parametrize("dist,param", [("u32", 0), ("mod100", 0), ("const", 0), ("lowbits", 9), ("lowbits", 12),
                                        ("lowbits", 23), ("sorted", 0), ("reversed", 0)])
def test_tile_sort(ls, oracle, torch_gpu, key, dist, param):
    """Every tile sorted; lowbits 12 / 23 put the varying bits across a digit boundary."""
    torch = torch_gpu
    T = ls.tile_keys()
    n = 5 * T + 1234
    a = oracle.gen(n, SEED + 3, dist, param=param)
    t = to_dev(torch, a)
    o = torch.empty_like(t)
    ls.tile_sort(t, o, n, key=key)
    torch.cuda.synchronize()
    got = from_dev(o)
    for s in range(0, n, T):
        np.testing.assert_array_equal(got[s:s + T], ref_sort(oracle, a[s:s + T].copy(), key))


# ---- digit histogram ----------------------------------------------------------------------
@pytest.mark.parametrize("bits", [8, 1])
@pytest.mark.parametrize("key", ["u32", "i32"])
def test_histogram(ls, oracle, torch_gpu, bits, key):
    torch = torch_gpu
    n = 1_000_003
    a = oracle.gen(n, SEED + 4, "u32")
    t = to_dev(torch, a)
    R, P = 1 << bits, (32 + bits - 1) // bits
    h = torch.zeros(P * R, dtype=torch.int32, device="cuda")
    ls.histogram(t, n, h, bits=bits, key=key)
    torch.cuda.synchronize()
    got = from_dev(h).reshape(P, R)
    x = a ^ np.uint32(0x80000000) if key == "i32" else a
    for p in range(P):
        d = (x >> np.uint32(p * bits)) & np.uint32(R - 1)
        np.testing.assert_array_equal(got[p], np.bincount(d, minlength=R).astype(np.uint32))


# ---- whole sorts ----------------------------------------------------------------------------
SIZES = [1, 2, 63, 64, 65, 1000, 8191, 8192, 8193, 32767, 32768, 32769, 65536, 100_000, (1 << 20) + 12345]
DISTS = ["u32", "u31", "mod100", "mod1000", "sorted", "reversed", "const", "lowbits"]


@pytest.mark.parametrize("algo", ["radix", "merge"])
@pytest.mark.parametrize("key", ["u32", "i32"])
@pytest.mark.parametrize("n", SIZES)
def test_sort_device_uniform(ls, oracle, torch_gpu, algo, key, n):
    torch = torch_gpu
    a = oracle.gen(n, SEED + 5 + n, "u32")
    t = to_dev(torch, a)
    o = torch.empty_like(t)
    ls.sort_device(t, o, n, key=key, algo=algo)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(from_dev(o), ref_sort(oracle, a, key))
    np.testing.assert_array_equal(from_dev(t), a)  # input untouched


@pytest.mark.parametrize("algo", ["radix", "merge", "radix-onesweep"])
@pytest.mark.parametrize("dist", DISTS)
@pytest.mark.parametrize("inplace", [False, True])
def test_sort_device_distributions(ls, oracle, torch_gpu, monkeypatch, algo, dist, inplace):
    """radix-onesweep: the onesweep passes at this size (LABSORT_RADIX_IMPL=onesweep): a
    constant input (no active pass: pass 0's launch copies it; in place: nothing to do),
    one or two active passes in place (the final copy) and the segmented plans."""
    torch = torch_gpu
    if algo == "radix-onesweep":
        monkeypatch.setenv("LABSORT_RADIX_IMPL", "onesweep")
        algo = "radix"
    n = 300_007
    a = oracle.gen(n, SEED + 6, dist, param=(0xABCDEF if dist == "const" else 11))
    for key in ("u32", "i32"):
        t = to_dev(torch, a)
        o = t if inplace else torch.empty_like(t)
        ls.sort_device(t, o, n, key=key, algo=algo)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(from_dev(o), ref_sort(oracle, a, key), err_msg=f"{key}")


@pytest.mark.parametrize("n", [1000, 8193, 70_000])
@pytest.mark.parametrize("key", ["u32", "i32"])
def test_sort_device_radix1(ls, oracle, torch_gpu, n, key):
    """letra.pdf's literal form: 32 one-bit split passes."""
    torch = torch_gpu
    a = oracle.gen(n, SEED + 7, "u32")
    t = to_dev(torch, a)
    o = torch.empty_like(t)
    ls.sort_device(t, o, n, key=key, algo="radix1")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(from_dev(o), ref_sort(oracle, a, key))


def test_sort_device_offsets_unaligned(ls, oracle, torch_gpu):
    """Sub-tensor views (pointer not 16-B aligned) go through the scalar paths."""
    torch = torch_gpu
    n = 200_001
    a = oracle.gen(n + 3, SEED + 8, "u32")
    t = to_dev(torch, a)
    o = torch.zeros_like(t)
    for algo in ("radix", "merge"):
        ls.sort_device(t[1:1 + n], o[3:3 + n - 2], n - 2, algo=algo)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(from_dev(o)[3:3 + n - 2], oracle.sort_u32(a[1:n - 1]))


@pytest.mark.parametrize("n", [(1 << 17), (1 << 17) + 1, 3 * 32768 + 7, (1 << 19) + 32768 * 3 + 5, (1 << 21) - 1,
                               (1 << 22) + 65536 + 128, (1 << 24) + 5])
@pytest.mark.parametrize("dist", ["u32", "lowbits2", "sorted", "reversed"])
def test_merge_four_way_shapes(ls, oracle, torch_gpu, n, dist):
    """The merge sort's four-way passes (merge4.hip): run counts that leave the last group
    with one to three runs, short last runs, the first four-way pass over 32768-key runs
    (the rank kernel's per-sample path: fewer samples per run than a workgroup takes) and
    later ones (its bracketed path), keys repeated across every run (block cuts inside
    runs of equal keys), int32 order."""
    torch = torch_gpu
    base = "lowbits" if dist == "lowbits2" else dist
    a = oracle.gen(n, SEED + 40 + n % 997, base, param=2 if dist == "lowbits2" else 0)  # lowbits2: keys 0..3
    t = to_dev(torch, a)
    o = torch.empty_like(t)
    for key in ("u32", "i32"):
        ls.sort_device(t, o, n, key=key, algo="merge")
        torch.cuda.synchronize()
        np.testing.assert_array_equal(from_dev(o), ref_sort(oracle, a, key), err_msg=f"{key}")


@pytest.mark.parametrize("m", list(range(1, 17)))
def test_merge_four_way_short_last_run(ls, oracle, torch_gpu, m):
    """n = m * 32768 + L for L in {1, 127, 128, 129}: the last group of every four-way pass
    (runs of 32768, 65536, 131072 keys, after a pairwise pass or not) ends in a run of one
    key, just under / exactly / just over one sample stride (M4_S = 128), at each of the four
    run positions as m varies, with the group's later runs empty: the rank kernel's sample
    counts and the cut rounds' clamps (merge4.hip m4_cut_round) at their edges."""
    torch = torch_gpu
    for L in (1, 127, 128, 129):
        n = m * 32768 + L
        a = oracle.gen(n, SEED + 60 + m * 7 + L, "u32")
        t = to_dev(torch, a)
        o = torch.empty_like(t)
        for key in ("u32", "i32"):
            ls.sort_device(t, o, n, key=key, algo="merge")
            torch.cuda.synchronize()
            np.testing.assert_array_equal(from_dev(o), ref_sort(oracle, a, key), err_msg=f"n={n} {key}")


# ---- merge building blocks ------------------------------------------------------------------
def test_merge_pass(ls, oracle, torch_gpu):
    torch = torch_gpu
    run = 8192
    n = 5 * run + 777
    a = oracle.gen(n, SEED + 9, "mod1000")
    runs = np.concatenate([oracle.sort_u32(a[s:s + run]) for s in range(0, n, run)])
    t = to_dev(torch, runs)
    o = torch.empty_like(t)
    part = torch.empty(ls.merge_parts(n), dtype=torch.int32, device="cuda")
    ls.merge_pass(t, o, n, run, part)
    torch.cuda.synchronize()
    got = from_dev(o)
    for s in range(0, n, 2 * run):
        np.testing.assert_array_equal(got[s:s + 2 * run], oracle.sort_u32(a[s:s + 2 * run]))


@pytest.mark.parametrize("la,lb", [(0, 5000), (5000, 0), (1, 1), (70_000, 30_001), (4096, 4096)])
def test_merge_diagonal_ranges(ls, oracle, torch_gpu, la, lb):
    """merge-split step of the multi-GPU exchange: a diagonal range of merge(A,B)."""
    torch = torch_gpu
    A = oracle.sort_u32(oracle.gen(la, SEED + 10, "mod1000"))
    B = oracle.sort_u32(oracle.gen(lb, SEED + 11, "mod1000"))
    tA = to_dev(torch, A) if la else torch.empty(1, dtype=torch.int32, device="cuda")
    tB = to_dev(torch, B) if lb else torch.empty(1, dtype=torch.int32, device="cuda")
    tot = la + lb
    for d0, d1 in [(0, tot), (0, tot // 2), (tot // 2, tot), (tot // 3, tot // 3 + 5000)]:
        d1 = min(d1, tot)
        if d1 <= d0:
            continue
        out = torch.empty(d1 - d0, dtype=torch.int32, device="cuda")
        part = torch.empty(ls.merge_parts(d1 - d0), dtype=torch.int32, device="cuda")
        ls.merge(tA, la, tB, lb, out, d0, d1, part)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(from_dev(out), oracle.merge_split(A, B, d0, d1))


@pytest.mark.parametrize("lens", [
    [5000, 7000],                                  # K = 2
    [1, 0, 3, 2],                                  # tiny and empty runs, K = 4
    [100_000, 99_999, 1, 0, 65_536, 70_001, 512, 4096],  # K = 8, ragged
    [300_000, 0, 0, 0, 0],                         # one non-empty run of five (K = 8)
    [40_000] * 3,                                  # three equal runs (K = 4, one empty)
    [1 << 18] * 8,                                 # eight equal runs
])
@pytest.mark.parametrize("dist,key", [("mod1000", "u32"), ("u32", "i32"), ("const", "u32"), ("u32", "u32")])
def test_merge_runs(ls, oracle, torch_gpu, lens, dist, key):
    """K-way merge of the runs one rank receives in the multi-GPU exchange (and of the
    merge sort's passes): equals std::sort of the concatenation, base offset > 0."""
    torch = torch_gpu
    base = 37
    n = sum(lens)
    a = oracle.gen(n, SEED + 20 + len(lens), dist)
    offs, pos, runs = [base], base, []
    for q, L in enumerate(lens):
        runs.append(ref_sort(oracle, a[pos - base:pos - base + L], key))
        pos += L
        offs.append(pos)
    buf = np.concatenate([np.zeros(base, np.uint32)] + runs + [np.zeros(5, np.uint32)])
    t = to_dev(torch, buf)
    o = torch.full_like(t, 12345)
    ls.merge_runs(t, o, offs, key=key)
    torch.cuda.synchronize()
    got = from_dev(o)
    np.testing.assert_array_equal(got[base:base + n], ref_sort(oracle, a, key))
    assert (got[:base] == 12345).all() and (got[base + n:] == 12345).all()


def test_merge_runs_bad_args(ls, torch_gpu):
    torch = torch_gpu
    t = torch.zeros(16, dtype=torch.int32, device="cuda")
    with pytest.raises(ls.LabsortError):
        ls.merge_runs(t, t, [0, 8, 16])            # in place
    with pytest.raises(ls.LabsortError):
        ls.merge_runs(t, torch.zeros_like(t), [0, 9, 8])  # decreasing offsets
    with pytest.raises(ls.LabsortError):
        ls.merge_runs(t, torch.zeros_like(t), list(range(11)))  # 10 runs > 8


# ---- key/value (sort_by_key) ----------------------------------------------------
@pytest.mark.parametrize("algo", ["radix", "merge"])
@pytest.mark.parametrize("n", [1, 100, 16384, 16385, 100_003, (1 << 20) + 7, 3_000_017])
@pytest.mark.parametrize("dist,key", [("u32", "u32"), ("mod100", "i32"), ("const", "u32"), ("u32", "i32"),
                                      ("lowbits", "u32")])
def test_sort_pairs(ls, oracle, torch_gpu, n, dist, key, algo):
    """Stable: equal keys keep input order, so the payload (the input index) must equal
    std::stable_sort's permutation exactly."""
    torch = torch_gpu
    k = oracle.gen(n, SEED + 30, dist, param=5)
    v = np.arange(n, dtype=np.uint32) * np.uint32(2654435761)  # payloads: a bijection of the index
    ek, ev = oracle.stable_sort_pairs(k, v, key)
    tk, tv = to_dev(torch, k), to_dev(torch, v)
    ok, ov = torch.full_like(tk, -1), torch.full_like(tv, -1)
    ls.sort_pairs_device(tk, tv, ok, ov, n, key=key, algo=algo)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(from_dev(ok), ek)
    np.testing.assert_array_equal(from_dev(ov), ev)
    np.testing.assert_array_equal(from_dev(tk), k)  # input untouched
    # fully in place
    ls.sort_pairs_device(tk, tv, tk, tv, n, key=key, algo=algo)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(from_dev(tk), ek)
    np.testing.assert_array_equal(from_dev(tv), ev)


@pytest.mark.parametrize("algo", ["radix", "merge"])
@pytest.mark.parametrize("dist", ["u32", "sorted", "reversed", "lowbits"])
def test_sort_pairs_large(ls, oracle, torch_gpu, dist, algo):
    """Key/value at 2^24 + 5 pairs. radix: the persistent onesweep passes (segmented
    look-back chains, partial first tiles per segment) carrying the payloads; merge: the
    key/value four-way passes (k_m4_merge_kv; lowbits: 32 distinct keys, so block cuts fall
    inside long runs of equal keys and stability is what decides the payload order)."""
    torch = torch_gpu
    n = (1 << 24) + 5
    k = oracle.gen(n, SEED + 31, dist, param=5 if dist == "lowbits" else 0)
    v = np.arange(n, dtype=np.uint32)
    ek, ev = oracle.stable_sort_pairs(k, v, "u32")
    tk, tv = to_dev(torch, k), to_dev(torch, v)
    ok, ov = torch.empty_like(tk), torch.empty_like(tv)
    ls.sort_pairs_device(tk, tv, ok, ov, n, key="u32", algo=algo)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(from_dev(ok), ek)
    np.testing.assert_array_equal(from_dev(ov), ev)


def test_sort_pairs_bad_args(ls, torch_gpu):
    torch = torch_gpu
    t = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    u = torch.zeros_like(t)
    o = torch.zeros_like(t)
    with pytest.raises(ls.LabsortError):
        ls.sort_pairs_device(t, u, t, o, t.numel())   # keys in place, payloads not
    with pytest.raises(ls.LabsortError):
        ls.sort_pairs_device(t, u, o, o, t.numel())   # keys and payloads to one buffer
    with pytest.raises(ls.LabsortError):
        ls.sort_pairs_device(t, u, o, t, t.numel(), workspace=torch.zeros(16, dtype=torch.uint8, device="cuda"))


# ---- host-pointer drop-ins (lab.h) ------------------------------------------------------------
@pytest.mark.parametrize("n", [256, 1024, 65536, 1 << 17, 1 << 20])
def test_order_array_matches_std_sort(ls, oracle, torch_gpu, n):
    a = oracle.gen(n, SEED + 12, "mod100").astype(np.int32)  # main.cpp:10 data shape
    b = a.copy()
    ls.order_array(b)
    np.testing.assert_array_equal(b, np.sort(a))


def test_order_array_negative_keys(ls, oracle, torch_gpu):
    """Outside the reference's domain (F6: it hangs); we sort signed order."""
    a = oracle.gen(100_000, SEED + 13, "u32").view(np.int32).copy()
    b = a.copy()
    ls.order_array(b)
    np.testing.assert_array_equal(b, np.sort(a))


@pytest.mark.parametrize("symbol", ["sort", "_Z11order_arrayPii"])
@pytest.mark.parametrize("n", [1000, 65536, (1 << 20) + 3])
def test_c_abi_sort_symbols_match_std_sort(ls, oracle, torch_gpu, symbol, n):
    """The exported entry points themselves, called through ctypes as a C caller would:
    the north_star's extern "C" sort(int*, int) and order_array(int*, int) (lab.h:9),
    signed int keys, against std::sort in int32 order (the oracle)."""
    import ctypes
    a = oracle.gen(n, SEED + 16, "u32").view(np.int32).copy()
    b = a.copy()
    fn = getattr(ls.lib, symbol)
    fn.restype = None
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    fn(b.ctypes.data, n)
    np.testing.assert_array_equal(b, oracle.sort_i32(a))


def test_order_with_trust(ls, oracle):
    a = oracle.gen(65536, SEED + 14, "mod1000").astype(np.int32)
    b = a.copy()
    ls.order_with_trust(b)
    np.testing.assert_array_equal(b, np.sort(a))


@pytest.mark.parametrize("algo", ["radix", "merge", "radix1"])
def test_sort_host_algorithms(ls, oracle, torch_gpu, algo):
    a = oracle.gen(123_457, SEED + 15, "u32")
    b = a.copy()
    ls.sort_host(b, algo=algo)
    np.testing.assert_array_equal(b, oracle.sort_u32(a))


@pytest.mark.parametrize("n,off", [(1, 0), (4095, 0), (16384 * 3 + 5, 0), ((1 << 22) + 7, 0), (100_001, 1)])
def test_copy(ls, oracle, torch_gpu, n, off):
    """labsort_copy (the bench's copy ceiling): 16-B tiles, word tail, unaligned views"""
    torch = torch_gpu
    a = oracle.gen(n + off, SEED + 77, "u32")
    t = to_dev(torch, a)
    o = torch.zeros(n + 2, dtype=torch.int32, device="cuda")
    ls.copy(t[off:], o[1 if off else 0:], n)
    torch.cuda.synchronize()
    got = from_dev(o)
    np.testing.assert_array_equal(got[(1 if off else 0):(1 if off else 0) + n], a[off:])


def test_count_descents(ls, oracle, torch_gpu):
    torch = torch_gpu
    a = np.arange(10_000, dtype=np.uint32)
    a[[10, 500, 9000]] = 0
    t = to_dev(torch, a)
    c = torch.zeros(1, dtype=torch.int32, device="cuda")
    ls.count_descents(t, a.size, c)
    torch.cuda.synchronize()
    assert int(c.item()) == 3


@pytest.mark.parametrize("impl", ["gather", "onesweep"])
def test_timing_hooks(ls, oracle, torch_gpu, monkeypatch, impl):
    torch = torch_gpu
    monkeypatch.setenv("LABSORT_RADIX_IMPL", impl)
    n = 1 << 20
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    ls.fill(t, n, SEED, "u32")
    o = torch.empty_like(t)
    ls.timing_enable(True)
    ls.sort_device(t, o, n, algo="radix")
    torch.cuda.synchronize()
    ms, cnt = ls.timing_read({"gather": "gsweep", "onesweep": "onesweep"}[impl])
    ms2, cnt2 = ls.timing_read("gcopy")
    ls.timing_enable(False)
    # four 8-bit passes (gather: pass 0 always runs, 1-3 active here)
    assert cnt == 4 and ms > 0
    assert cnt2 == (1 if impl == "gather" else 0)


# ---- segmented look-back chains: pass structure edge cases ----------------------------
@pytest.mark.parametrize("mask,name", [
    (0xFFFF00FF, "trivial middle pass (byte 1 constant)"),
    (0x0F0F0F0F, "every digit in nibble group 0 (one segment holds all keys)"),
    (0xFF0000FF, "two trivial middle passes"),
    (0xF0F0F0F0, "every digit's low nibble zero"),
    (0x000000FF, "one active pass"),
    (0x80000001, "sign bit + bit 0 only"),
])
@pytest.mark.parametrize("key", ["u32", "i32"])
@pytest.mark.parametrize("n", [8192 * 16 + 5, (1 << 21) + 777])
@pytest.mark.parametrize("impl", ["", "onesweep"])
def test_sort_device_pass_structure(ls, oracle, torch_gpu, monkeypatch, mask, name, key, n, impl):
    torch = torch_gpu
    if impl:
        monkeypatch.setenv("LABSORT_RADIX_IMPL", impl)
    a = oracle.gen(n, SEED + 16, "u32") & np.uint32(mask)
    t = to_dev(torch, a)
    o = torch.empty_like(t)
    ls.sort_device(t, o, n, key=key, algo="radix")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(from_dev(o), ref_sort(oracle, a, key), err_msg=name)


OSP_TILE = 16384   # k_onesweep_p tile (csrc/common.h OSP_TILE)
NSEG = 16         # position segments of the first pass (common.h NSEG)


def _boundary_sizes():
    ts = 32768    # labsort_tile_keys(): sizes up to it take the LDS tile-sort path
    return sorted({1, 100, ts - 1, ts, ts + 1, ts + 100, 2 * OSP_TILE + 1, NSEG * OSP_TILE - 1,
                   NSEG * OSP_TILE, NSEG * OSP_TILE + 1, 3 * NSEG * OSP_TILE + OSP_TILE // 2 + 1})


@pytest.mark.parametrize("n", _boundary_sizes())
def test_sort_device_segment_boundaries(ls, oracle, torch_gpu, n):
    """Sizes around the 16 position segments x 16384-key tiles of the first onesweep
    pass, and just above the tile-sort small path (the smallest multi-tile look-back
    chains)."""
    torch = torch_gpu
    assert ls.tile_keys() == 32768
    a = oracle.gen(n, SEED + 17 + n, "u32")
    t = to_dev(torch, a)
    ls.sort_device(t, t, n, algo="radix")
    torch.cuda.synchronize()
    np.testing.assert_array_equal(from_dev(t), oracle.sort_u32(a))


@pytest.mark.parametrize("algo", ["radix", "merge"])
@pytest.mark.parametrize("pairs", [False, True])
def test_workspace_status_reports_device_error(ls, oracle, torch_gpu, pairs, algo):
    """A sort that a kernel flagged (radix: the look-back spin limit; merge: a four-way
    block with inconsistent cuts, skipped) is reported as LABSORT_ERR_DEVICE by
    labsort_workspace_status, never as OK; the next sort on the workspace clears the word.
    The error word is the workspace's first word in both layouts."""
    torch = torch_gpu
    n = 1 << 20
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    ls.fill(t, n, SEED + 40, "u32")
    o = torch.empty_like(t)
    if pairs:
        v, vo = torch.arange(n, dtype=torch.int32, device="cuda"), torch.empty_like(t)
        ws = torch.empty(ls.pairs_workspace_bytes(n, algo), dtype=torch.uint8, device="cuda")
        run = lambda: ls.sort_pairs_device(t, v, o, vo, n, algo=algo, workspace=ws)  # noqa: E731
        status = lambda: ls.pairs_workspace_status(ws, n, algo)  # noqa: E731
    else:
        ws = torch.empty(ls.workspace_bytes(n, algo), dtype=torch.uint8, device="cuda")
        run = lambda: ls.sort_device(t, o, n, algo=algo, workspace=ws)  # noqa: E731
        status = lambda: ls.workspace_status(ws, n, algo)  # noqa: E731
    run()
    status()  # clean sort: OK
    ws[:4].view(torch.int32).fill_(1)  # what the kernels' error store leaves behind
    with pytest.raises(ls.LabsortError, match="device-side"):
        status()
    run()
    status()
    np.testing.assert_array_equal(from_dev(o), oracle.sort_u32(oracle.gen(n, SEED + 40, "u32")))
