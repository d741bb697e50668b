"""labsort_sort_host_multi / labsort_sort_host_ranks (csrc/multi.hip) on the GPU:
the whole one-process multi-GPU schedule -- shard H2D, local sorts, splitters, cut
points, exchange, K-way merge of the received runs, D2H to global offsets -- with
p ranks sharing cuda:0 and exchanging by peer copies, checked against std::sort (the
oracle).  The RCCL transport is exercised with one rank (its send to itself goes
through ncclSend/ncclRecv in a group); its multi-device use needs an 8-GPU node
(unmeasured on hardware here)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("p", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("dist,key", [("u32", "u32"), ("mod100", "i32"), ("const", "u32"), ("u32", "i32")])
@pytest.mark.parametrize("n", [5, 100_003, 1 << 21])
def test_sort_host_ranks_peer(ls, oracle, torch_gpu, p, dist, key, n):
    a = oracle.gen(n, 0x5EED7200 + n + p, dist)
    exp = oracle.sort_i32(a.view(np.int32)).view(np.uint32) if key == "i32" else oracle.sort_u32(a)
    b = a.view(np.int32).copy() if key == "i32" else a.copy()
    ls.sort_host_ranks(b, [0] * p, transport="peer")
    np.testing.assert_array_equal(b.view(np.uint32), exp)
    t, sent = ls.multi_timing()
    assert t["total"] > 0 and sent <= n * 4


def test_sort_host_ranks_balance_const(ls, oracle, torch_gpu):
    """a constant array is split evenly (ranges are contiguous global ranks)"""
    n, p = 1 << 22, 8
    b = np.full(n, 7, dtype=np.uint32)
    ls.sort_host_ranks(b, [0] * p, transport="peer")
    assert np.all(b == 7)
    _, sent = ls.multi_timing()
    assert sent <= (n // p) * 4 * 1.05  # a rank sends at most about its share


@pytest.mark.parametrize("n", [1, 1 << 16, (1 << 22) + 3])
def test_sort_host_multi_one_gpu(ls, oracle, torch_gpu, n):
    a = oracle.gen(n, 0x5EED7300 + n, "u32")
    b = a.copy()
    ls.sort_host_multi(b, 1)
    np.testing.assert_array_equal(b, oracle.sort_u32(a))


def test_sort_host_ranks_rccl_one_rank(ls, oracle, torch_gpu):
    """RCCL transport (dlopen'd librccl, ncclCommInitAll, grouped send/recv)."""
    n = (1 << 20) + 11
    a = oracle.gen(n, 0x5EED7400, "u32")
    b = a.copy()
    ls.sort_host_ranks(b, [0], transport="rccl")
    np.testing.assert_array_equal(b, oracle.sort_u32(a))


def test_sort_host_multi_arg_checks(ls, torch_gpu):
    torch = torch_gpu
    a = np.zeros(16, np.uint32)
    ndev = torch.cuda.device_count()
    with pytest.raises(ls.LabsortError):
        ls.sort_host_multi(a, ndev + 1)  # more ranks than devices
    with pytest.raises(ls.LabsortError):
        ls.sort_host_ranks(a, [0, 0], transport="rccl")  # RCCL: one rank per device
    with pytest.raises(ls.LabsortError):
        ls.sort_host_ranks(a, [0] * 9, transport="peer")  # > LABSORT_MULTI_MAX_RANKS
