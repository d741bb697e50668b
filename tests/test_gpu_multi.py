"""labsort_sort_host_multi / labsort_sort_host_ranks (csrc/multi.hip) on the GPU:
the whole one-process multi-GPU schedule (csrc/dist_plan.h) -- chunked shard H2D under
the chunk sorts, splitters, cut points, exchange, merge of the received runs, D2H to
global offsets range by range -- with p ranks sharing cuda:0 and exchanging by peer
copies, checked against std::sort (the oracle) and, at BASELINE config 5's size (2^30
keys in 8 ranks), against the SHA-256 fixture.  The RCCL transport's multi-device use
needs an 8-GPU node (unmeasured on hardware here); ncclCommInitAll with one rank runs."""
import hashlib
import json
import os

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
    # the plan's work and wait (time inside its collectives), every rank's arrival times
    assert t["plan_work"] >= 0 and t["plan_wait"] >= 0
    for c in ls.multi_collectives(p):
        for k in ("samples", "counts"):
            assert 0 <= c[k][0] <= c[k][1]
        assert c["samples"][1] <= c["counts"][0]


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


@pytest.mark.parametrize("phase", ["local_sort", "bounds", "recv", "exchange"])
def test_sort_host_ranks_rank_failure(ls, oracle, torch_gpu, phase):
    """one in-process rank failing (ls.test_fault, the schedule's test hook; "exchange": it
    leaves without taking part) ends the call with that rank's own error
    (LABSORT_ERR_DEVICE), not a hang; the next call works"""
    import time
    a = oracle.gen(300_000, 0x5EED7500, "u32")
    ls.test_fault(phase, 2)
    try:
        t0 = time.monotonic()
        with pytest.raises(ls.LabsortError) as e:
            ls.sort_host_ranks(a.copy(), [0] * 4, transport="peer")
        assert e.value.status == ls.ERR_DEVICE
        assert time.monotonic() - t0 < 30
    finally:
        ls.test_fault(None)
    b = a.copy()
    ls.sort_host_ranks(b, [0] * 4, transport="peer")
    np.testing.assert_array_equal(b, oracle.sort_u32(a))


def test_sort_host_ranks_rccl_one_rank_fault(ls, oracle, torch_gpu):
    """the RCCL transport (nonblocking communicators, bounded waits): a rank failing at its
    local sort returns its error, the communicators are recreated and the next call works"""
    a = oracle.gen((1 << 18) + 3, 0x5EED7401, "u32")
    ls.test_fault("local_sort", 0)
    try:
        with pytest.raises(ls.LabsortError) as e:
            ls.sort_host_ranks(a.copy(), [0], transport="rccl")
        assert e.value.status == ls.ERR_DEVICE
    finally:
        ls.test_fault(None)
    b = a.copy()
    ls.sort_host_ranks(b, [0], transport="rccl")
    np.testing.assert_array_equal(b, oracle.sort_u32(a))


def test_test_fault_rejects_unknown_phase(ls):
    with pytest.raises(ls.LabsortError) as e:
        ls.test_fault("nonsense", 0)
    assert e.value.status == ls.ERR_ARG
    ls.test_fault(None)


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


@pytest.mark.parametrize("p", [1, 3, 8])
@pytest.mark.parametrize("pin", ["0", "1"])
def test_sort_host_ranks_chunked(ls, oracle, torch_gpu, monkeypatch, p, pin):
    """Each rank's shard copied and sorted in 8 chunks (LABSORT_HOST_PIPE=1 chunks from
    2^16 keys per rank), with and without the caller's array page-locked (LABSORT_PIN)."""
    monkeypatch.setenv("LABSORT_HOST_PIPE", "1")
    monkeypatch.setenv("LABSORT_PIN", pin)
    n = p * ((1 << 19) + 77)
    a = oracle.gen(n, 0x5EED7500 + p, "u32")
    b = a.copy()
    ls.sort_host_ranks(b, [0] * p, transport="peer")
    np.testing.assert_array_equal(b, oracle.sort_u32(a))
    t, _ = ls.multi_timing()
    assert t["h2d"] > 0 and t["local_sort"] > 0 and t["total"] > 0
    assert sum(ls.multi_range_counts(p)) == n


GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "big.json")


def test_config5_2e30_8ranks_one_gpu(ls, torch_gpu):
    """BASELINE config 5 at full size through its own partition: 2^30 uint32 keys, 8
    ranks (sharing cuda:0: peer copies stand in for xGMI), chunked H2D per rank,
    splitters, exchange, merge, ranged D2H; the result matches the fixture word for
    word and every rank's range is within 2 % of n/8."""
    torch = torch_gpu
    c = json.load(open(GOLD))["config5_2^30_u32"]
    n = 1 << c["log2n"]
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    ls.fill(t, n, c["seed"], c["dist"])
    a = t.cpu().numpy().view(np.uint32)
    del t
    torch.cuda.empty_cache()
    ls.sort_host_ranks(a, [0] * 8, transport="peer")
    counts = ls.multi_range_counts(8)
    assert sum(counts) == n and max(counts) <= 1.02 * n / 8, counts
    assert int(a[0]) == c["first"] and int(a[-1]) == c["last"] and int(a[n // 2]) == c["median"]
    assert hashlib.sha256(a.tobytes()).hexdigest() == c["sha256_sorted_u32"]
    ph, sent = ls.multi_timing()
    print("config5 8 ranks on one GPU:", {k: round(v, 2) for k, v in ph.items()}, "max sent", sent)
