"""The multi-GPU exchange plan of labsort_sort_host_multi (csrc/multi.hip) on host
shards, through the labsort_multi_plan test hook: the same splitter choice and cut
logic as the device path, with std::upper_bound standing in for the device bound
queries (no GPU).  Routing every piece by the plan, merging each rank's received
runs in rank order and concatenating the ranks must give the oracle's sort of the
whole array, and (key, rank, position) splitters keep every range near n/p even
when one key repeats everywhere."""
import numpy as np
import pytest


def route(ls, oracle, shards, key):
    order = (lambda a: a.view(np.int32)) if key == "i32" else (lambda a: a)
    shards = [np.sort(order(s.view(np.uint32)), kind="stable").view(np.uint32) for s in shards]
    cuts = ls.multi_plan(shards, key=key)
    p = len(shards)
    assert cuts.shape == (p, p + 1)
    ranges = []
    for r in range(p):
        c = cuts[r]
        assert c[0] == 0 and c[p] == shards[r].size and np.all(np.diff(c) >= 0)
    for j in range(p):
        got = np.concatenate([shards[i][cuts[i, j]:cuts[i, j + 1]] for i in range(p)])
        ranges.append(np.sort(order(got), kind="stable").view(np.uint32))
    return ranges


CASES = [("u32", "u32", 1), ("u32", "u32", 2), ("u32", "u32", 3), ("u32", "u32", 8), ("mod100", "u32", 8),
         ("const", "u32", 4), ("const", "u32", 8), ("u32", "i32", 8), ("mod1000", "i32", 5), ("sorted", "u32", 8),
         ("lowbits", "u32", 7)]


@pytest.mark.parametrize("dist,key,p", CASES)
@pytest.mark.parametrize("m", [1, 1000, 65_537])
def test_plan_routes_to_global_order(ls, oracle, dist, key, p, m):
    full = oracle.gen(m * p, 0x5EED7000 + p + m, dist, param=3 if dist == "lowbits" else 0)
    shards = [full[r * m:(r + 1) * m] for r in range(p)]
    ranges = route(ls, oracle, shards, key)
    got = np.concatenate(ranges)
    exp = oracle.sort_i32(full.view(np.int32)).view(np.uint32) if key == "i32" else oracle.sort_u32(full)
    np.testing.assert_array_equal(got, exp)
    if m >= 1000:
        # every range within ~2 sample strides of its share, whatever the key repetition
        assert max(r.size for r in ranges) <= m * 1.02 + 2, [r.size for r in ranges]


def test_plan_ragged_and_empty_shards(ls, oracle):
    full = oracle.gen(10_000, 0x5EED7100, "mod100")
    sizes = [0, 3000, 0, 1, 6999, 0]
    shards, o = [], 0
    for s in sizes:
        shards.append(full[o:o + s])
        o += s
    got = np.concatenate(route(ls, oracle, shards, "u32"))
    np.testing.assert_array_equal(got, oracle.sort_u32(full))


def test_plan_rejects_bad_args(ls):
    with pytest.raises(ls.LabsortError):
        ls.multi_plan([np.zeros(4, np.uint32)] * 9)  # more than LABSORT_MULTI_MAX_RANKS
