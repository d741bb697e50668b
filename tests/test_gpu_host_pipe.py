"""The pipelined host-pointer sort (labsort_sort_host / order_array for n >= 2^27, forced
here from 2^16 with LABSORT_HOST_PIPE=1):
chunked H2D overlapped with the chunk sorts, two half merges, and the final merge by
diagonal ranges with each range's D2H started as it lands (api.hip, HOST_CHUNKS).
Checked bit-exact against std::sort (the oracle) and against the unpipelined path
(LABSORT_HOST_PIPE=0) on the same input; ragged sizes leave a short last chunk and
uneven halves."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED0700


def ref(oracle, a, key):
    return oracle.sort_i32(a.view(np.int32)).view(np.uint32) if key == "i32" else oracle.sort_u32(a)


def host(a, key):
    return a.view(np.int32) if key == "i32" else a


@pytest.mark.parametrize("n,dist,key,algo", [
    (1 << 24, "u32", "u32", "auto"),
    ((1 << 24) + 12345, "mod100", "i32", "radix"),
    (3 * (1 << 23) + 5, "u31", "i32", "merge"),
    ((1 << 24) + 7, "const", "u32", "auto"),
    ((1 << 25) - 3, "reversed", "i32", "auto"),
    (1 << 24, "sorted", "u32", "radix"),
    ((1 << 24) + 1, "lowbits", "u32", "radix"),
])
def test_pipelined_host_sort(ls, oracle, torch_gpu, monkeypatch, n, dist, key, algo):
    a = oracle.gen(n, SEED + n % 97, dist, param=5 if dist == "lowbits" else (9 if dist == "const" else 0))
    exp = ref(oracle, a, key)
    monkeypatch.setenv("LABSORT_HOST_PIPE", "1")  # the pipeline below its default threshold (2^27)
    b = a.copy()
    ls.sort_host(host(b, key), algo=algo)
    np.testing.assert_array_equal(b, exp)
    monkeypatch.setenv("LABSORT_HOST_PIPE", "0")
    c = a.copy()
    ls.sort_host(host(c, key), algo=algo)
    np.testing.assert_array_equal(c, exp)


def test_pipelined_host_sort_back_to_back(ls, oracle, torch_gpu, monkeypatch):
    """the cached buffers and events are reused: a second call with other keys must not
    see the first call's data (Y is rewritten only after the previous D2H copies)"""
    monkeypatch.setenv("LABSORT_HOST_PIPE", "1")
    n = (1 << 24) + 333
    for s in range(3):
        a = oracle.gen(n, SEED + 50 + s, ("u32", "mod1000", "u31")[s])
        b = a.copy()
        ls.sort_host(b, algo="auto")
        np.testing.assert_array_equal(b, oracle.sort_u32(a))


@pytest.mark.parametrize("n", [1 << 16, (1 << 16) + 5, 100_003])
def test_pipelined_host_sort_small_chunks(ls, oracle, torch_gpu, monkeypatch, n):
    """chunks at and below the tile-sort small path (the chunk sorts take other paths)"""
    monkeypatch.setenv("LABSORT_HOST_PIPE", "1")
    a = oracle.gen(n, SEED + 7, "u32")
    b = a.copy()
    ls.sort_host(b, algo="radix")
    np.testing.assert_array_equal(b, oracle.sort_u32(a))
