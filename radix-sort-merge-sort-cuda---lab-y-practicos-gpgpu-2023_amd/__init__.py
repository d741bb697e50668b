"""labsort -- MI355X-native (gfx950) integer sort behind the reference's order_array API.

The product is the native library `liblabsort.so` (HIP kernels + C++ host
orchestration, C-ABI in include/labsort.h).  This module is a thin ctypes view of
it for Python callers, tests and bench.py:

  order_array(a)          lab.h:9 / lab.cu:303  -- int32 numpy array sorted in place
                          through the GPU (host pointer, synchronous)
  order_with_trust(a)     lab.h:10 / lab.cu:404 -- thrust::sort on the host pointer
  sort_device(...)        the device-pointer sort (keys already in HBM)
  wave_tile_sort, tile_sort, merge_pass, merge, histogram  -- the building blocks

There is no CPU fallback: if the shared library is missing this module raises
at import, and every device call raises LabsortError on a failed status.
The package directory name is not a Python identifier; import it with
``importlib.import_module("radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd")``.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# LABSORT_LIBRARY: path of an alternative build (diagnostic builds under harness/exp)
LIB_PATH = os.environ.get("LABSORT_LIBRARY") or os.path.join(HERE, "liblabsort.so")

OK, ERR_ARG, ERR_HIP, ERR_DEVICE, ERR_PEER = 0, 1, 2, 3, 4
ALGO = {"radix": 0, "merge": 1, "radix1": 2, "auto": 3}
KEY = {"u32": 0, "i32": 1}
DIST = {"u32": 0, "u31": 1, "mod100": 2, "mod1000": 3, "sorted": 4, "reversed": 5, "const": 6, "lowbits": 7}
KCLASS = {"histogram": 0, "onesweep": 1, "tile_sort": 2, "merge": 3, "partition": 4, "gsweep": 5, "gcopy": 6,
          "copy": 7, "merge4": 8}

# exported symbols of include/labsort.h + lab.h (checked by tests/test_abi.py)
C_SYMBOLS = [
    "labsort_version", "labsort_error_string", "labsort_last_hip_error", "labsort_hip_error_string",
    "labsort_max_keys", "labsort_tile_keys", "labsort_merge_tile_keys", "labsort_workspace_bytes",
    "labsort_sort_device", "labsort_sort_host", "labsort_wave_tile_sort", "labsort_tile_sort",
    "labsort_merge_parts", "labsort_merge_pass", "labsort_merge", "labsort_histogram", "labsort_fill",
    "labsort_count_descents", "labsort_timing_enable", "labsort_timing_read", "labsort_upper_bound", "sort",
    "labsort_merge_runs_workspace_bytes", "labsort_merge_runs",
    "labsort_pair_tile_keys", "labsort_pairs_workspace_bytes", "labsort_sort_pairs_device",
    "labsort_workspace_status", "labsort_pairs_workspace_status",
    "labsort_sort_host_multi", "labsort_sort_host_ranks", "labsort_multi_timing", "labsort_multi_last_hip_error",
    "labsort_multi_plan", "labsort_multi_error_detail", "labsort_multi_range_counts",
    "labsort_comm_unique_id", "labsort_comm_init_rccl", "labsort_comm_init_host", "labsort_comm_destroy",
    "labsort_dist_sort", "labsort_dist_timing", "labsort_dist_last_hip_error",
    "labsort_multi_collectives", "labsort_dist_collectives", "labsort_copy",
    "labsort_comm_set_timeout", "labsort_test_fault",
]
XFER = {"auto": 0, "rccl": 1, "peer": 2}
MULTI_PHASES = ["h2d", "local_sort", "plan", "exchange", "merge", "d2h", "total", "plan_work", "plan_wait"]
COLLECTIVES = ["samples", "counts", "grow"]  # the schedule's collectives, in order (labsort.h)
CXX_SYMBOLS = ["_Z11order_arrayPii", "_Z16order_with_trustPii"]


class LabsortError(RuntimeError):
    """A failed LABSORT_* status; .status holds the code (ERR_ARG, ERR_HIP, ERR_DEVICE,
    ERR_PEER)."""

    def __init__(self, msg: str, status: int = 0):
        super().__init__(msg)
        self.status = status


# labsort_host_coll (include/labsort.h): host collectives supplied by the caller
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
ALLTOALLV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t),
                                ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t))


class HostColl(ctypes.Structure):
    _fields_ = [("ctx", ctypes.c_void_p), ("allgather", ALLGATHER_FN), ("alltoallv", ALLTOALLV_FN)]


def host_coll(obj) -> HostColl:
    """labsort_host_coll whose callbacks call obj.allgather(h_in, h_out, nbytes) and
    obj.alltoallv(h_send, send_bytes, h_recv, recv_bytes) (raw host addresses and lists
    of byte counts).  A Python exception in a callback becomes a failed status.  Keep
    the returned structure alive while the communicator uses it."""
    import traceback

    def ag(_ctx, h_in, h_out, nbytes):
        try:
            obj.allgather(h_in, h_out, int(nbytes))
            return 0
        except Exception:
            traceback.print_exc()
            return 1

    def a2a(_ctx, h_send, sb, h_recv, rb):
        try:
            n = obj.world
            obj.alltoallv(h_send, [int(sb[i]) for i in range(n)], h_recv, [int(rb[i]) for i in range(n)])
            return 0
        except Exception:
            traceback.print_exc()
            return 1

    return HostColl(None, ALLGATHER_FN(ag), ALLTOALLV_FN(a2a))


def _load() -> ctypes.CDLL:
    # One HIP runtime per process: torch ships its own libamdhip64.so (SONAME
    # libamdhip64.so.7).  Loading torch first makes liblabsort's DT_NEEDED
    # libamdhip64.so.7 bind to that already-loaded runtime, so torch tensors and
    # our kernels share one device context.  Loaded the other way round, a second
    # runtime would come up and find no device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the labsort path has no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    p, sz, i, u64 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_uint64
    L.labsort_version.restype = ctypes.c_char_p
    L.labsort_error_string.restype = ctypes.c_char_p
    L.labsort_error_string.argtypes = [i]
    L.labsort_hip_error_string.restype = ctypes.c_char_p
    L.labsort_hip_error_string.argtypes = [i]
    for f in ("labsort_max_keys", "labsort_workspace_bytes"):
        getattr(L, f).restype = sz
    L.labsort_max_keys.argtypes = [i]
    L.labsort_tile_keys.restype = sz
    L.labsort_merge_tile_keys.restype = sz
    L.labsort_merge_parts.restype = sz
    L.labsort_merge_parts.argtypes = [sz]
    L.labsort_workspace_bytes.argtypes = [sz, i]
    L.labsort_sort_device.argtypes = [p, p, sz, i, i, p, sz, p]
    L.labsort_sort_host.argtypes = [p, sz, i, i]
    L.labsort_wave_tile_sort.argtypes = [p, sz, i, p]
    L.labsort_tile_sort.argtypes = [p, p, sz, i, p]
    L.labsort_merge_pass.argtypes = [p, p, sz, sz, i, p, p]
    L.labsort_merge.argtypes = [p, sz, p, sz, p, sz, sz, i, p, p]
    L.labsort_merge_runs_workspace_bytes.restype = sz
    L.labsort_merge_runs_workspace_bytes.argtypes = [sz]
    L.labsort_merge_runs.argtypes = [p, p, ctypes.POINTER(sz), i, i, p, sz, p]
    L.labsort_pair_tile_keys.restype = sz
    L.labsort_pair_tile_keys.argtypes = []
    L.labsort_pairs_workspace_bytes.restype = sz
    L.labsort_pairs_workspace_bytes.argtypes = [sz, i]
    L.labsort_sort_pairs_device.argtypes = [p, p, p, p, sz, i, i, p, sz, p]
    L.labsort_workspace_status.argtypes = [p, sz, i, p]
    L.labsort_sort_host_multi.argtypes = [p, sz, i, i]
    L.labsort_sort_host_ranks.argtypes = [p, sz, i, i, p, i]
    L.labsort_multi_timing.argtypes = [ctypes.POINTER(ctypes.c_double), i, ctypes.POINTER(sz)]
    L.labsort_multi_plan.argtypes = [ctypes.POINTER(p), ctypes.POINTER(sz), i, i, ctypes.POINTER(sz)]
    L.labsort_multi_range_counts.argtypes = [ctypes.POINTER(sz), i]
    L.labsort_multi_error_detail.restype = ctypes.c_char_p
    L.labsort_multi_error_detail.argtypes = []
    L.labsort_comm_unique_id.argtypes = [p]
    L.labsort_comm_init_rccl.argtypes = [ctypes.POINTER(p), p, i, i]
    L.labsort_comm_init_host.argtypes = [ctypes.POINTER(p), i, i, ctypes.POINTER(HostColl)]
    L.labsort_comm_destroy.argtypes = [p]
    L.labsort_comm_set_timeout.argtypes = [p, ctypes.c_double]
    L.labsort_test_fault.argtypes = [ctypes.c_char_p, i]
    L.labsort_dist_sort.argtypes = [p, p, sz, i, p, ctypes.POINTER(p), ctypes.POINTER(sz), ctypes.POINTER(sz)]
    L.labsort_dist_timing.argtypes = [p, ctypes.POINTER(ctypes.c_double), i, ctypes.POINTER(sz)]
    L.labsort_dist_last_hip_error.argtypes = [p]
    L.labsort_multi_collectives.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), i, i]
    L.labsort_dist_collectives.argtypes = [p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), i]
    L.labsort_copy.argtypes = [p, p, sz, p]
    L.labsort_pairs_workspace_status.argtypes = [p, sz, i, p]
    L.labsort_histogram.argtypes = [p, sz, i, i, p, p]
    L.labsort_fill.argtypes = [p, sz, u64, i, u64, u64, p]
    L.labsort_count_descents.argtypes = [p, sz, i, p, p]
    L.labsort_upper_bound.argtypes = [p, sz, i, p, sz, p, p]
    L.labsort_timing_enable.argtypes = [i]
    L.labsort_timing_read.argtypes = [i, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong)]
    L.sort.argtypes = [p, i]
    L.sort.restype = None
    fn = getattr(L, "_Z11order_arrayPii")
    fn.argtypes = [p, i]
    fn.restype = None
    fn = getattr(L, "_Z16order_with_trustPii")
    fn.argtypes = [p, i]
    fn.restype = None
    return L


lib = _load()


def version() -> str:
    return lib.labsort_version().decode()


def _check(status: int, what: str) -> None:
    if status != OK:
        msg = lib.labsort_error_string(status).decode()
        if status == ERR_HIP:
            msg += ": " + lib.labsort_hip_error_string(lib.labsort_last_hip_error()).decode()
        raise LabsortError(f"{what} failed: {msg}", status)


def _ptr(x) -> int:
    """Device or host address of a torch tensor / numpy array / int."""
    if isinstance(x, int):
        return x
    if isinstance(x, np.ndarray):
        assert x.flags["C_CONTIGUOUS"]
        return x.ctypes.data
    assert x.is_contiguous()
    return x.data_ptr()


def _stream(stream) -> int | None:
    if stream is None:
        try:
            import torch
            if torch.cuda.is_available():
                return torch.cuda.current_stream().cuda_stream
        except Exception:
            pass
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


# ---- host-pointer drop-ins (lab.h) -------------------------------------------------
def order_array(a: np.ndarray) -> None:
    """Sort an int32 numpy array in place on the GPU (lab.cu:303 semantics).

    Unlike the C++ drop-in, which prints GPUassert and exits, this raises."""
    assert a.dtype == np.int32 and a.flags["C_CONTIGUOUS"]
    _check(lib.labsort_sort_host(a.ctypes.data, a.size, KEY["i32"], _default_algo()), "order_array")


def sort_host(a: np.ndarray, algo: str = "radix") -> None:
    """Sort a uint32 or int32 numpy array in place through the GPU."""
    key = "i32" if a.dtype == np.int32 else "u32"
    assert a.dtype in (np.int32, np.uint32) and a.flags["C_CONTIGUOUS"]
    _check(lib.labsort_sort_host(a.ctypes.data, a.size, KEY[key], ALGO[algo]), "sort_host")


def order_with_trust(a: np.ndarray) -> None:
    """thrust::sort on the host pointer (lab.cu:404): rocThrust's sequential CPU sort."""
    assert a.dtype == np.int32 and a.flags["C_CONTIGUOUS"]
    getattr(lib, "_Z16order_with_trustPii")(a.ctypes.data, a.size)


def _check_multi(status: int, what: str) -> None:
    if status != OK:
        detail = lib.labsort_multi_error_detail().decode()
        raise LabsortError(f"{what} failed: {lib.labsort_error_string(status).decode()}"
                           + (f" ({detail})" if detail else ""), status)


def sort_host_multi(a: np.ndarray, ngpus: int) -> None:
    """Sort a uint32/int32 numpy array in place across devices 0..ngpus-1 of this
    process (labsort_sort_host_multi: per-GPU shards, RCCL splitter exchange)."""
    key = "i32" if a.dtype == np.int32 else "u32"
    assert a.dtype in (np.int32, np.uint32) and a.flags["C_CONTIGUOUS"]
    _check_multi(lib.labsort_sort_host_multi(a.ctypes.data, a.size, KEY[key], ngpus), "sort_host_multi")


def sort_host_ranks(a: np.ndarray, devices, transport: str = "auto") -> None:
    """As sort_host_multi with an explicit rank -> device map (ranks may share a
    device with transport "peer": the whole schedule on one GPU)."""
    key = "i32" if a.dtype == np.int32 else "u32"
    assert a.dtype in (np.int32, np.uint32) and a.flags["C_CONTIGUOUS"]
    dv = (ctypes.c_int * len(devices))(*devices)
    _check_multi(lib.labsort_sort_host_ranks(a.ctypes.data, a.size, KEY[key], len(devices), dv, XFER[transport]),
                 "sort_host_ranks")


def multi_timing() -> tuple[dict, int]:
    """Phase times (ms) of the last multi-GPU host sort and the most key bytes one
    rank sent to its peers."""
    ms = (ctypes.c_double * len(MULTI_PHASES))()
    sent = ctypes.c_size_t(0)
    _check(lib.labsort_multi_timing(ms, len(MULTI_PHASES), ctypes.byref(sent)), "multi_timing")
    return dict(zip(MULTI_PHASES, list(ms))), sent.value


def multi_collectives(nranks: int) -> list:
    """Per rank of the last multi-GPU host sort: {collective: (arrive_ms, leave_ms)} on the
    host clock since that rank's start (-1: the collective did not run)."""
    k = len(COLLECTIVES)
    a, b = (ctypes.c_double * (nranks * k))(), (ctypes.c_double * (nranks * k))()
    _check(lib.labsort_multi_collectives(a, b, nranks, k), "multi_collectives")
    return [{COLLECTIVES[c]: (a[r * k + c], b[r * k + c]) for c in range(k)} for r in range(nranks)]


def multi_range_counts(nranks: int) -> list:
    """Keys of each rank's range of the sorted array in the last multi-GPU host sort."""
    c = (ctypes.c_size_t * nranks)()
    _check(lib.labsort_multi_range_counts(c, nranks), "multi_range_counts")
    return list(c)


def multi_plan(shards, key: str = "u32") -> np.ndarray:
    """Cut points of the multi-GPU exchange plan for sorted host shards (test hook):
    cuts[r, j] = first position of the piece rank r sends to rank j (cuts[r, p] = m_r)."""
    arrs = [np.ascontiguousarray(x).view(np.uint32) for x in shards]
    p = len(arrs)
    ptrs = (ctypes.c_void_p * p)(*[x.ctypes.data if x.size else None for x in arrs])
    ms = (ctypes.c_size_t * p)(*[x.size for x in arrs])
    cuts = (ctypes.c_size_t * (p * (p + 1)))()
    _check(lib.labsort_multi_plan(ptrs, ms, p, KEY[key], cuts), "multi_plan")
    return np.array(list(cuts), dtype=np.int64).reshape(p, p + 1)


def test_fault(phase: str | None, rank: int = -1) -> None:
    """TEST HOOK (labsort_test_fault): rank `rank` of the following multi-GPU sorts of this
    process fails at `phase` ("local_sort", "bounds", "recv", "grow", "exchange"); None
    disarms.  The product never arms it."""
    _check(lib.labsort_test_fault(phase.encode() if phase else None, rank), "test_fault")


def set_comm_timeout(seconds: float) -> None:
    """Deadline of every wait on the peers of the in-process RCCL transport and of the
    communicators created afterwards (labsort_comm_set_timeout(NULL, seconds))."""
    _check(lib.labsort_comm_set_timeout(None, float(seconds)), "comm_set_timeout")


class DistComm:
    """One rank's communicator of the distributed merge sort (labsort_comm_t; one
    process per GPU).  DistComm.rccl(world, rank, uid) over RCCL (uid from
    DistComm.unique_id() on rank 0, broadcast by the caller), or DistComm.host(world,
    rank, coll) over host collectives (an object with world, allgather and alltoallv:
    dist.GlooColl), which lets several ranks share one GPU in the tests."""

    def __init__(self, handle, keep=None):
        self.h = ctypes.c_void_p(handle)
        self._keep = keep

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        _check_multi(lib.labsort_comm_unique_id(buf), "labsort_comm_unique_id")
        return buf.raw

    @classmethod
    def rccl(cls, world: int, rank: int, uid: bytes) -> "DistComm":
        h = ctypes.c_void_p(0)
        ub = ctypes.create_string_buffer(bytes(uid), 128)
        _check_multi(lib.labsort_comm_init_rccl(ctypes.byref(h), ub, world, rank), "labsort_comm_init_rccl")
        return cls(h.value)

    @classmethod
    def host(cls, world: int, rank: int, coll_obj) -> "DistComm":
        coll = host_coll(coll_obj)
        h = ctypes.c_void_p(0)
        _check_multi(lib.labsort_comm_init_host(ctypes.byref(h), world, rank, ctypes.byref(coll)),
                     "labsort_comm_init_host")
        return cls(h.value, keep=(coll, coll_obj))

    def sort(self, d_keys, m: int, key: str = "u32", stream=None) -> tuple[int, int, int]:
        """labsort_dist_sort: (device address, count, global offset) of this rank's range
        of the sorted array, valid until the next sort on this communicator."""
        res, cnt, goff = ctypes.c_void_p(0), ctypes.c_size_t(0), ctypes.c_size_t(0)
        st = lib.labsort_dist_sort(self.h, _ptr(d_keys) if m else None, m, KEY[key], _stream(stream),
                                   ctypes.byref(res), ctypes.byref(cnt), ctypes.byref(goff))
        _check_multi(st, "labsort_dist_sort")
        return res.value or 0, cnt.value, goff.value

    def sort_tensor(self, d_keys, m: int, key: str = "u32", stream=None, copy: bool = True):
        """As sort(), with the range as an int32 torch tensor and its global offset.  By
        default the range is copied out of the communicator's buffer; copy=False returns a
        zero-copy view of that buffer instead, which keeps this communicator alive but is
        INVALID after its next sort: that sort may overwrite the buffer, or free it and
        allocate a larger one (a range that outgrew it), leaving the view on freed memory."""
        ptr, cnt, goff = self.sort(d_keys, m, key, stream)
        v = self.view(ptr, cnt, owner=self)
        return (v.clone() if copy else v), goff

    @staticmethod
    def view(ptr: int, count: int, owner=None):
        """int32 torch tensor on the current device viewing `count` keys at device
        address `ptr` (__cuda_array_interface__; no copy).  `owner` (e.g. the DistComm whose
        buffer it is) is kept alive as long as the tensor."""
        import torch
        if count == 0:
            return torch.empty(0, dtype=torch.int32, device="cuda")

        class _View:
            __cuda_array_interface__ = {"shape": (count,), "typestr": "<i4", "data": (ptr, False), "version": 2,
                                        "strides": None}
        holder = _View()
        holder.owner = owner
        t = torch.as_tensor(holder, device="cuda")
        t._labsort_owner = holder  # the buffer's owner lives as long as the tensor
        return t

    def set_timeout(self, seconds: float) -> None:
        """Deadline of this communicator's waits on its peers (RCCL; labsort_comm_set_timeout)."""
        _check(lib.labsort_comm_set_timeout(self.h, float(seconds)), "comm_set_timeout")

    def timing(self) -> tuple[dict, int]:
        ms = (ctypes.c_double * len(MULTI_PHASES))()
        sent = ctypes.c_size_t(0)
        _check(lib.labsort_dist_timing(self.h, ms, len(MULTI_PHASES), ctypes.byref(sent)), "dist_timing")
        return dict(zip(MULTI_PHASES, list(ms))), sent.value

    def collectives(self) -> dict:
        """{collective: (arrive_ms, leave_ms)} of this rank's last sort (-1: not run)."""
        k = len(COLLECTIVES)
        a, b = (ctypes.c_double * k)(), (ctypes.c_double * k)()
        _check(lib.labsort_dist_collectives(self.h, a, b, k), "dist_collectives")
        return {COLLECTIVES[c]: (a[c], b[c]) for c in range(k)}

    def close(self) -> None:
        if self.h.value:
            _check_multi(lib.labsort_comm_destroy(self.h), "labsort_comm_destroy")
            self.h = ctypes.c_void_p(0)

    def __del__(self):
        try:
            if self.h.value:
                lib.labsort_comm_destroy(self.h)
        except Exception:
            pass


def _default_algo() -> int:
    """as the C++ drop-ins: LABSORT_ALGO names the algorithm, else "auto" (merge up to
    LABSORT_AUTO_MERGE_MAX_KEYS keys, radix above)"""
    return ALGO.get(os.environ.get("LABSORT_ALGO", "auto"), ALGO["auto"])


# ---- device API (torch tensors or raw device addresses) ----------------------------
def workspace_bytes(n: int, algo: str = "radix") -> int:
    return int(lib.labsort_workspace_bytes(n, ALGO[algo]))


GS_MIN_N, GS_MAX_N = 1 << 16, 1 << 25  # LABSORT_ALGO_RADIX's gathered-pass window (common.h)


def radix_impl(n: int) -> str:
    """Which LSD implementation LABSORT_ALGO_RADIX runs for n keys: "gather" (gsweep.hip)
    or "onesweep" (kernels.hip), as api.hip's use_gather decides."""
    env = os.environ.get("LABSORT_RADIX_IMPL", "")
    if env == "gather":
        return "gather"
    if GS_MIN_N <= n < GS_MAX_N and env != "onesweep":
        return "gather"
    return "onesweep"


def max_keys(algo: str = "radix") -> int:
    return int(lib.labsort_max_keys(ALGO[algo]))


def tile_keys() -> int:
    return int(lib.labsort_tile_keys())


def merge_tile_keys() -> int:
    return int(lib.labsort_merge_tile_keys())


def merge_parts(n: int) -> int:
    return int(lib.labsort_merge_parts(n))


def sort_device(d_in, d_out, n: int, key: str = "u32", algo: str = "radix", workspace=None,
                workspace_bytes_: int | None = None, stream=None) -> None:
    """Sort n keys d_in -> d_out (may alias) asynchronously on `stream`.

    With a caller-owned `workspace` the call stays asynchronous; check the kernels'
    own error report with workspace_status() once the result is needed.  Without
    one, the call allocates a workspace, synchronises and checks it itself."""
    own = workspace is None
    if own:
        import torch
        workspace = torch.empty(max(workspace_bytes(n, algo), 1), dtype=torch.uint8, device="cuda")
    wsb = workspace_bytes_ if workspace_bytes_ is not None else (
        workspace.numel() * workspace.element_size() if hasattr(workspace, "numel") else workspace_bytes(n, algo))
    _check(lib.labsort_sort_device(_ptr(d_in), _ptr(d_out), n, KEY[key], ALGO[algo], _ptr(workspace), wsb,
                                   _stream(stream)), "sort_device")
    if own:
        workspace_status(workspace, n, algo, stream)


def workspace_status(workspace, n: int, algo: str = "radix", stream=None) -> None:
    """Synchronise `stream` and raise LabsortError(device-side error) if a kernel of the
    last sort_device(n, algo) on `workspace` reported a failure (labsort_workspace_status)."""
    _check(lib.labsort_workspace_status(_ptr(workspace), n, ALGO[algo], _stream(stream)), "sort_device (status)")


def pairs_workspace_status(workspace, n: int, algo: str = "radix", stream=None) -> None:
    """As workspace_status, for the last sort_pairs_device(n, algo) on `workspace`."""
    _check(lib.labsort_pairs_workspace_status(_ptr(workspace), n, ALGO[algo], _stream(stream)),
           "sort_pairs_device (status)")


def wave_tile_sort(d_keys, n: int, key: str = "u32", stream=None) -> None:
    _check(lib.labsort_wave_tile_sort(_ptr(d_keys), n, KEY[key], _stream(stream)), "wave_tile_sort")


def tile_sort(d_in, d_out, n: int, key: str = "u32", stream=None) -> None:
    _check(lib.labsort_tile_sort(_ptr(d_in), _ptr(d_out), n, KEY[key], _stream(stream)), "tile_sort")


def merge_pass(d_in, d_out, n: int, run: int, d_part, key: str = "u32", stream=None) -> None:
    _check(lib.labsort_merge_pass(_ptr(d_in), _ptr(d_out), n, run, KEY[key], _ptr(d_part), _stream(stream)),
           "merge_pass")


def merge(d_a, la: int, d_b, lb: int, d_out, d0: int, d1: int, d_part, key: str = "u32", stream=None) -> None:
    _check(lib.labsort_merge(_ptr(d_a) if la else 0, la, _ptr(d_b) if lb else 0, lb, _ptr(d_out), d0, d1,
                             KEY[key], _ptr(d_part), _stream(stream)), "merge")


def merge_runs_workspace_bytes(n: int) -> int:
    return int(lib.labsort_merge_runs_workspace_bytes(n))


def merge_runs(d_in, d_out, offsets, key: str = "u32", workspace=None, stream=None) -> None:
    """K-way merge (K <= 8) of the sorted runs d_in[offsets[q]:offsets[q+1]] into
    d_out[offsets[0]:offsets[-1]] (stable: equal keys keep run order)."""
    offs = [int(x) for x in offsets]
    if workspace is None:
        import torch
        workspace = torch.empty(max(merge_runs_workspace_bytes(offs[-1]), 1), dtype=torch.uint8, device="cuda")
    wsb = workspace.numel() * workspace.element_size()
    arr = (ctypes.c_size_t * len(offs))(*offs)
    _check(lib.labsort_merge_runs(_ptr(d_in), _ptr(d_out), arr, len(offs) - 1, KEY[key], _ptr(workspace), wsb,
                                  _stream(stream)), "merge_runs")


def pairs_workspace_bytes(n: int, algo: str = "radix") -> int:
    return int(lib.labsort_pairs_workspace_bytes(n, ALGO[algo]))


def pair_tile_keys() -> int:
    return int(lib.labsort_pair_tile_keys())


def sort_pairs_device(d_keys_in, d_vals_in, d_keys_out, d_vals_out, n: int, key: str = "u32", algo: str = "radix",
                      workspace=None, stream=None) -> None:
    """Stable sort of n (key, 4-byte payload) pairs (sort_by_key); equal keys keep
    their input order.  algo: "radix", "merge" or "auto".  Asynchronous on `stream`."""
    own = workspace is None
    if own:
        import torch
        workspace = torch.empty(max(pairs_workspace_bytes(n, algo), 1), dtype=torch.uint8, device="cuda")
    wsb = workspace.numel() * workspace.element_size()
    _check(lib.labsort_sort_pairs_device(_ptr(d_keys_in), _ptr(d_vals_in), _ptr(d_keys_out), _ptr(d_vals_out), n,
                                         KEY[key], ALGO[algo], _ptr(workspace), wsb, _stream(stream)),
           "sort_pairs_device")
    if own:
        pairs_workspace_status(workspace, n, algo, stream)


def histogram(d_keys, n: int, d_hist, bits: int = 8, key: str = "u32", stream=None) -> None:
    _check(lib.labsort_histogram(_ptr(d_keys), n, KEY[key], bits, _ptr(d_hist), _stream(stream)), "histogram")


def fill(d_out, n: int, seed: int, dist: str = "u32", param: int = 0, first: int = 0, stream=None) -> None:
    if dist == "reversed" and param == 0:
        param = first + n
    _check(lib.labsort_fill(_ptr(d_out), n, seed & (2**64 - 1), DIST[dist], param, first, _stream(stream)),
           "fill")


def upper_bound(d_sorted, n: int, d_values, nv: int, d_out, key: str = "u32", stream=None) -> None:
    """d_out[i] = number of keys <= d_values[i] in the sorted run (key order)."""
    _check(lib.labsort_upper_bound(_ptr(d_sorted) if n else 0, n, KEY[key], _ptr(d_values), nv, _ptr(d_out),
                                   _stream(stream)), "upper_bound")


def copy(d_in, d_out, n: int, stream=None) -> None:
    """d_out[0..n) = d_in[0..n) (32-bit words) by the library's streaming copy kernel."""
    _check(lib.labsort_copy(_ptr(d_in), _ptr(d_out), n, _stream(stream)), "copy")


def count_descents(d_keys, n: int, d_count, key: str = "u32", stream=None) -> None:
    _check(lib.labsort_count_descents(_ptr(d_keys), n, KEY[key], _ptr(d_count), _stream(stream)),
           "count_descents")


def timing_enable(on: bool = True) -> None:
    _check(lib.labsort_timing_enable(1 if on else 0), "timing_enable")


def timing_read(kclass: str) -> tuple[float, int]:
    ms, cnt = ctypes.c_double(0.0), ctypes.c_longlong(0)
    _check(lib.labsort_timing_read(KCLASS[kclass], ctypes.byref(ms), ctypes.byref(cnt)), "timing_read")
    return ms.value, cnt.value
