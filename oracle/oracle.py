"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes view of oracle/liboracle.so (std::sort spec oracle, the counter-based
generator and the lane-level restatement of the reference's lab.cu).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module; the product package never does.

Pinning: parity unpinned by reference artifacts -- the reference ships no tests,
golden vectors or validated outputs, and its lab.cu is CUDA-only (no nvcc here;
a HIP build would need stand-in CUDA headers), so it cannot be run to produce
any.  The oracle is pinned instead by (1) the uniqueness of a keys-only ascending
sort (std::sort = the specification of order_array, letra.pdf p.3), checked
against numpy's sort and the committed fixtures in tests/golden/, and (2) the
lane-level restatement of lab.cu (labcu_restate.c), which reproduces the
reference's own results, including its failure modes F4/F5/F6.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

# LABCU_* status codes of labcu_restate.c
OK, LAUNCH_FAIL, HANG, UB, BAD_ARG = 0, 1, 2, 3, 4
STATUS_NAMES = {OK: "ok", LAUNCH_FAIL: "launch_fail", HANG: "hang", UB: "ub", BAD_ARG: "bad_arg"}

# generator distributions (same codes as include/labsort.h LABSORT_DIST_*)
DIST = {"u32": 0, "u31": 1, "mod100": 2, "mod1000": 3, "sorted": 4, "reversed": 5, "const": 6, "lowbits": 7}

_lib = None

# labsort_host_coll of include/labsort.h (the same layout as the package's HostColl)
_AG = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
_A2A = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t),
                        ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t))


class _HostColl(ctypes.Structure):
    _fields_ = [("ctx", ctypes.c_void_p), ("allgather", _AG), ("alltoallv", _A2A)]


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u64, p = ctypes.c_uint64, ctypes.c_void_p
        L.oracle_fill.argtypes = [p, u64, u64, ctypes.c_int, u64, u64]
        L.oracle_sort_u32.argtypes = [p, u64]
        L.oracle_sort_i32.argtypes = [p, u64]
        L.oracle_par_sort_u32.argtypes = [p, u64, ctypes.c_int]
        L.oracle_is_sorted_u32.argtypes = [p, u64]
        L.oracle_merge_split_u32.argtypes = [p, u64, p, u64, p, u64, u64]
        L.oracle_stable_sort_pairs.argtypes = [p, p, u64, ctypes.c_uint32]
        L.oracle_time_sort_u32.argtypes = [p, u64, ctypes.c_int, ctypes.c_int, p]
        L.oracle_time_sort_u32.restype = ctypes.c_double
        L.labcu_order_array.argtypes = [p, ctypes.c_int, ctypes.c_int]
        L.labcu_radix_tiles.argtypes = [p, ctypes.c_int]
        L.labcu_warp_scan.argtypes = [p]
        L.labcu_bsearch.argtypes = [p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_dist_sort.argtypes = [p, u64, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_HostColl),
                                       p, u64, ctypes.POINTER(u64), ctypes.POINTER(u64)]
        L.oracle_test_fault.argtypes = [ctypes.c_char_p, ctypes.c_int]
        L.oracle_test_fault.restype = None
        _lib = L
    return _lib


def _ptr(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


def gen(n: int, seed: int, dist: str = "u32", param: int = 0, first: int = 0) -> np.ndarray:
    """Counter-based keys first..first+n of stream (seed, dist) as uint32."""
    out = np.empty(n, dtype=np.uint32)
    if dist == "reversed" and param == 0:
        param = first + n
    lib().oracle_fill(_ptr(out), n, seed & (2**64 - 1), DIST[dist], param, first)
    return out


def sort_u32(a: np.ndarray) -> np.ndarray:
    out = np.ascontiguousarray(a, dtype=np.uint32).copy()
    lib().oracle_sort_u32(_ptr(out), out.size)
    return out


def sort_i32(a: np.ndarray) -> np.ndarray:
    out = np.ascontiguousarray(a, dtype=np.int32).copy()
    lib().oracle_sort_i32(_ptr(out), out.size)
    return out


def stable_sort_pairs(keys: np.ndarray, vals: np.ndarray, key: str = "u32"):
    """(keys, vals) stably sorted by key (std::stable_sort): the sort_by_key spec."""
    k = np.ascontiguousarray(keys).view(np.uint32).copy()
    v = np.ascontiguousarray(vals).view(np.uint32).copy()
    assert k.size == v.size
    lib().oracle_stable_sort_pairs(_ptr(k), _ptr(v), k.size, 0x80000000 if key == "i32" else 0)
    return k, v


def merge_split(a: np.ndarray, b: np.ndarray, lo: int, hi: int) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint32)
    b = np.ascontiguousarray(b, dtype=np.uint32)
    out = np.empty(hi - lo, dtype=np.uint32)
    lib().oracle_merge_split_u32(_ptr(a), a.size, _ptr(b), b.size, _ptr(out), lo, hi)
    return out


def labcu_order_array(a: np.ndarray, fix_f5: bool = False):
    """Run the lab.cu restatement; returns (status_name, output int32 array)."""
    out = np.ascontiguousarray(a, dtype=np.int32).copy()
    st = lib().labcu_order_array(_ptr(out), out.size, 1 if fix_f5 else 0)
    return STATUS_NAMES[st], out


def labcu_radix_tiles(a: np.ndarray):
    out = np.ascontiguousarray(a, dtype=np.int32).copy()
    st = lib().labcu_radix_tiles(_ptr(out), out.size)
    return STATUS_NAMES[st], out


def labcu_warp_scan(v: np.ndarray) -> np.ndarray:
    out = np.ascontiguousarray(v, dtype=np.int32).copy()
    assert out.size == 32
    lib().labcu_warp_scan(_ptr(out))
    return out


def labcu_bsearch(arr: np.ndarray, start: int, size: int, x: int, before_equal: bool) -> int:
    a = np.ascontiguousarray(arr, dtype=np.int32)
    return lib().labcu_bsearch(_ptr(a), start, size, x, 1 if before_equal else 0)


def time_sort_u32(keys: np.ndarray, threads: int = 1, reps: int = 1) -> float:
    """Seconds for `reps` CPU sorts of private copies of `keys` (copy untimed)."""
    keys = np.ascontiguousarray(keys, dtype=np.uint32)
    scratch = np.empty_like(keys)
    return lib().oracle_time_sort_u32(_ptr(keys), keys.size, threads, reps, _ptr(scratch))


def test_fault(phase: str | None, rank: int = -1) -> None:
    """Arm (phase, rank) -- "local_sort", "bounds", "recv", "grow" or "exchange" -- or
    disarm (None) the schedule's test failure for the following dist_sort calls."""
    lib().oracle_test_fault(phase.encode() if phase else None, rank)


def dist_sort(shard: np.ndarray, key: str, world: int, rank: int, coll, cap: int = 0) -> tuple[np.ndarray, int]:
    """One rank of the PRODUCT's multi-GPU schedule (csrc/dist_plan.h, dist::sort_rank)
    with host rank operations (std::sort, std::upper_bound, std::merge) over `coll`'s
    host collectives (world, allgather(h_in, h_out, nbytes), alltoallv(h_send,
    send_bytes, h_recv, recv_bytes): the package's dist.GlooColl).  Returns this rank's
    range of the sorted array and its global offset.  cap: room for the range (default
    twice the shard times the world size; pass the global key count for ragged shards)."""
    import traceback

    def ag(_c, hi, ho, nb):
        try:
            coll.allgather(hi, ho, int(nb))
            return 0
        except Exception:
            traceback.print_exc()
            return 1

    def a2a(_c, hs, sb, hr, rb):
        try:
            coll.alltoallv(hs, [int(sb[i]) for i in range(world)], hr, [int(rb[i]) for i in range(world)])
            return 0
        except Exception:
            traceback.print_exc()
            return 1

    hc = _HostColl(None, _AG(ag), _A2A(a2a))
    a = np.ascontiguousarray(shard).view(np.uint32)
    cap = cap or 2 * a.size * world + 16
    out = np.empty(cap, dtype=np.uint32)
    cnt, goff = ctypes.c_uint64(0), ctypes.c_uint64(0)
    st = lib().oracle_dist_sort(_ptr(a) if a.size else None, a.size, 1 if key == "i32" else 0, world, rank,
                                ctypes.byref(hc), _ptr(out), cap, ctypes.byref(cnt), ctypes.byref(goff))
    if st != 0:
        raise RuntimeError(f"oracle_dist_sort: status {st}")
    return out[:cnt.value].copy(), goff.value
