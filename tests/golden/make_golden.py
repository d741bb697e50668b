"""tests/golden/make_golden.py -- regenerate the committed golden fixtures.

    python tests/golden/make_golden.py

The reference ships no tests, golden vectors or validated outputs,
and its CUDA sources cannot be built or run here (no nvcc, no GPU).  A keys-only
ascending sort has exactly one correct output, so the fixtures pin:

  small.npz   inputs from the counter-based generator for
              n in 32..4096 and four distributions, their std::sort output, and
              what the lane-level restatement of lab.cu (oracle/labcu_restate.c)
              returns for the same input: status + output + ref_correct flag
              (documents where the reference's own result equals std::sort, and
              the F5 / F6 failure modes);
  f5.npz      the smallest F5 counter-example found (n = 2^11, 31-bit keys): the
              reference's wrong output and the fixed pipeline's correct output;
  big.json    SHA-256 of the generator's input and of the std::sort output for
              the BASELINE.json configs (2^16, 2^20, 2^28) and a few more, so the
              GPU tests check full-size results word for word without a CPU sort.

Uses the oracle (test infrastructure) only.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import oracle as O  # noqa: E402

SMALL_N = [32, 64, 128, 256, 512, 1024, 2048, 4096]
SMALL_DISTS = ["u32", "u31", "mod100", "mod1000"]
BIG = [  # (name, log2n, seed, dist)
    ("config1_2^16_u32", 16, 0x5EED0001, "u32"),
    ("config2_2^20_u32", 20, 0x5EED0002, "u32"),
    ("config2_2^20_u31", 20, 0x5EED0002, "u31"),
    ("2^24_u32", 24, 0x5EED0004, "u32"),
    ("2^24_mod1000", 24, 0x5EED0004, "mod1000"),
    ("config3_2^28_u32", 28, 0x5EED0003, "u32"),
    ("config5_2^30_u32", 30, 0x5EED0005, "u32"),
]


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    O.build()
    if len(sys.argv) > 2 and sys.argv[1] == "--big":
        return add_big(sys.argv[2:])
    small = {}
    for di, dist in enumerate(SMALL_DISTS):
        for n in SMALL_N:
            seed = 0x5EED1000 + 16 * di + n.bit_length()
            a = O.gen(n, seed, dist)
            key = f"{dist}_{n}"
            small[f"in_{key}"] = a
            small[f"sorted_{key}"] = O.sort_u32(a)
            small[f"sorted_i32_{key}"] = O.sort_i32(a.view(np.int32)).view(np.uint32)
            if dist == "u32":
                continue  # negative ints: the reference hangs (F6); tested separately
            st, out = O.labcu_order_array(a.view(np.int32))
            code = {v: k for k, v in O.STATUS_NAMES.items()}[st]
            small[f"ref_status_{key}"] = np.array([code], dtype=np.int32)
            small[f"ref_out_{key}"] = out.view(np.uint32)
    np.savez_compressed(os.path.join(HERE, "small.npz"), **small)

    # F5 counter-example: first seed at n = 2^11 (31-bit keys) the reference mis-sorts
    n = 1 << 11
    for s in range(1000):
        a = O.gen(n, 0x5EED5000 + s, "u31")
        st, out = O.labcu_order_array(a.view(np.int32))
        if st == "ok" and not np.array_equal(out.view(np.uint32), O.sort_u32(a)):
            st2, fixed = O.labcu_order_array(a.view(np.int32), fix_f5=True)
            assert st2 == "ok" and np.array_equal(fixed.view(np.uint32), O.sort_u32(a))
            np.savez_compressed(os.path.join(HERE, "f5.npz"), seed=np.array([0x5EED5000 + s], dtype=np.uint64),
                                inp=a, ref_out=out.view(np.uint32), fixed_out=fixed.view(np.uint32),
                                sorted=O.sort_u32(a))
            print("F5 counter-example seed", hex(0x5EED5000 + s))
            break
    else:
        raise SystemExit("no F5 counter-example found")

    add_big([name for name, *_ in BIG], fresh=True)


def add_big(names, fresh=False):
    """(Re)compute the big.json entries `names` (python make_golden.py --big NAME...)."""
    path = os.path.join(HERE, "big.json")
    big = {} if fresh else json.load(open(path))
    for name, lg, seed, dist in BIG:
        if name not in names:
            continue
        a = O.gen(1 << lg, seed, dist)
        b = a.copy()
        O.lib().oracle_par_sort_u32(b.ctypes.data, b.size, os.cpu_count() or 1)
        assert O.lib().oracle_is_sorted_u32(b.ctypes.data, b.size)
        big[name] = {"log2n": lg, "seed": seed, "dist": dist, "sha256_input": sha(a), "sha256_sorted_u32": sha(b),
                     "first": int(b[0]), "last": int(b[-1]), "median": int(b[b.size // 2])}
        if lg <= 24:
            c = a.view(np.int32).copy()
            c.sort(kind="stable")
        else:  # int32 order of the same multiset: the negative keys (top bit set) first
            k = int(np.searchsorted(b, np.uint32(1 << 31)))
            c = np.concatenate([b[k:], b[:k]])
        big[name]["sha256_sorted_i32"] = sha(c)
        del c
        print(name, big[name]["sha256_sorted_u32"][:16])
        del a, b
    with open(path, "w") as f:
        json.dump(big, f, indent=1)


if __name__ == "__main__":
    main()
