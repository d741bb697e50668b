"""Multi-GPU merge sort: one process per GPU, pairwise RCCL send/recv over xGMI.

The reference runs on one GPU only (run.sh:11); the north_star partitions n over
the GPUs of one node for the merge-sort path: every rank sorts its shard locally,
then a bitonic network of pairwise *merge-split* steps (Baudet & Stevenson's
block form of Batcher's network: compare-exchange replaced by "merge my block
with my partner's, keep the lower or the upper half") leaves rank r holding
global ranks [r*m, (r+1)*m) of the sorted array.  The merge-split step is the
reference's merge (lab.cu:144-182, A before B on ties) restricted to one half of
the output diagonal (`labsort_merge` with [0,m) or [m,2m)).

Each step exchanges shards with ONE partner over torch.distributed point-to-point
send/recv (backend "nccl" = RCCL on ROCm, one xGMI link per pair); log2(p)*(log2(p)+1)/2
steps for p ranks.  `partial=True` moves only the keys that cross: both sides
first swap a strided sample of their shards, bracket the split point, swap the
bracketing window, agree on the exact split k, then send k keys each way.

`dist_sort_splitters` is the all-link form (the default of bench.py) and a thin
caller of the product: labsort_dist_sort runs the schedule of csrc/dist_plan.h in C++
(the same code the one-process multi-GPU path and the oracle's CPU instantiation run):
every rank sorts its shard, the ranks agree on p-1 (key, rank, position) splitters
from a regular sample of every shard, cut their sorted shards at them, send piece j to
rank j with pairwise send/recv posted to all peers at once (all 7 xGMI links of a GPU
carry data together instead of one per step), and merge the p received runs in rank
order.  Communicators: RCCL (make_comm(backend="nccl"): ncclCommInitRank with rank 0's
unique id) or host-staged gloo collectives (GlooColl, tests).

For the bitonic network the local operations are pluggable (`Ops`): liblabsort.so on
the rank's GPU (`HipOps`), or numpy in the CPU tests, so that schedule is exercised
with the gloo backend on machines without GPUs.
Communication is pluggable too (`P2PComm` = torch.distributed; `HostStagedComm`
stages device tensors through host memory for a CPU backend in tests).
"""
from __future__ import annotations

import contextlib
import math
import time

import torch
import torch.distributed as dist


class Ops:
    """Local operations the exchange schedule needs (all keys int32-viewed uint32/int32)."""

    def local_sort(self, t: torch.Tensor, out_of_place: bool = False) -> torch.Tensor:
        """Sorted keys of t: in place, or into a new tensor when out_of_place."""
        raise NotImplementedError

    def merge(self, a: torch.Tensor, b: torch.Tensor, d0: int, d1: int) -> torch.Tensor:
        """elements d0..d1-1 of merge(a, b), a before b on ties"""
        raise NotImplementedError

    def key_le(self, x: int, y: int) -> bool:
        raise NotImplementedError

    def order(self, t: torch.Tensor) -> torch.Tensor:
        """int64 view of int32-stored keys that is monotone in key order"""
        f = 0x80000000 if getattr(self, "key", "u32") == "i32" else 0
        return (t.to(torch.int64) & 0xFFFFFFFF) ^ f


class HipOps(Ops):
    """liblabsort.so on the current GPU (local operations of the bitonic network)."""

    def __init__(self, ls, key: str = "u32", local_algo: str = "radix", stream=None):
        self.ls, self.key, self.algo, self.stream = ls, key, local_algo, stream
        self._ws = None
        self._part = None

    def _workspace(self, n):
        need = max(self.ls.workspace_bytes(n, self.algo), 256)
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device="cuda")
        return self._ws

    def local_sort(self, t, out_of_place=False):
        ws = self._workspace(t.numel())
        out = torch.empty_like(t) if out_of_place else t
        self.ls.sort_device(t, out, t.numel(), key=self.key, algo=self.algo, workspace=ws, stream=self.stream)
        # the kernels' own error report (a look-back spin that expired); synchronises
        self.ls.workspace_status(ws, t.numel(), self.algo, stream=self.stream)
        return out

    def merge(self, a, b, d0, d1):
        out = torch.empty(max(d1 - d0, 1), dtype=torch.int32, device=a.device if a.numel() else b.device)
        parts = self.ls.merge_parts(d1 - d0)
        if self._part is None or self._part.numel() < parts:
            self._part = torch.empty(parts, dtype=torch.int32, device=out.device)
        self.ls.merge(a, a.numel(), b, b.numel(), out, d0, d1, self._part, key=self.key, stream=self.stream)
        return out[: d1 - d0]

    def key_le(self, x, y):
        f = 0x80000000 if self.key == "i32" else 0
        return ((x & 0xFFFFFFFF) ^ f) <= ((y & 0xFFFFFFFF) ^ f)


class P2PComm:
    """Pairwise exchange over torch.distributed point-to-point ops (RCCL on the GPU
    box: one xGMI link per pair; gloo on CPU)."""

    def __init__(self, group=None):
        self.group = group
        self.sent_bytes = 0   # key bytes this rank sent over point-to-point ops
        self.p2p_rounds = 0   # exchange calls (one partner, or all peers at once)
        self.timed = False    # bench: synchronise around each exchange and add its wall time
        self.exchange_s = 0.0

    def _sync(self):
        if self.timed and torch.cuda.is_available():
            torch.cuda.synchronize()

    def exchange(self, send: torch.Tensor, recv: torch.Tensor, partner: int) -> None:
        self.sent_bytes += send.numel() * send.element_size()
        self.p2p_rounds += 1
        self._sync()
        t0 = time.perf_counter()
        g = self.group
        ops = [dist.P2POp(dist.isend, send, partner, group=g), dist.P2POp(dist.irecv, recv, partner, group=g)]
        for r in dist.batch_isend_irecv(ops):
            r.wait()
        self._sync()
        self.exchange_s += time.perf_counter() - t0


class HostStagedComm(P2PComm):
    """Test adapter: device tensors are staged through host memory and exchanged
    with a CPU backend (gloo), so the GPU-side schedule (HipOps on one device) can
    be exercised by several processes sharing one GPU."""

    def exchange(self, send, recv, partner):
        hs = send.cpu()
        hr = torch.empty_like(hs)
        super().exchange(hs, hr, partner)
        recv.copy_(hr)


def schedule(world: int):
    """(stage, step) pairs of the bitonic network over `world` ranks (power of two)."""
    stages = int(math.log2(world))
    return [(s, t) for s in range(stages) for t in range(s, -1, -1)]


def partner_and_side(rank: int, stage: int, step: int):
    partner = rank ^ (1 << step)
    ascending = ((rank >> (stage + 1)) & 1) == 0
    keep_low = (rank < partner) == ascending
    return partner, keep_low


def _split_count(ops: Ops, mine: torch.Tensor, partner: int, keep_low: bool, stride: int, comm) -> int:
    """Number k of keys that cross: the low side gives its top k, the high side its
    bottom k.  With L = low side's block and H = high side's block (both sorted, m
    keys), k = #H among the m smallest of L u H (L first on ties) = m - corank_L(m).
    Found with two small exchanges: a strided sample, then the bracketing window."""
    m = mine.numel()
    # predicate P(i) = L[i] <= H[m-1-i] is true then false; corank = first false i.
    # low side samples L[j*stride]; high side samples H[m-1-j*stride].
    idx = torch.arange(0, m, stride, device=mine.device)
    if keep_low:
        samp = mine[idx]
    else:
        samp = mine[(m - 1) - idx]
    other = torch.empty_like(samp)
    comm.exchange(samp.contiguous(), other, partner)
    Ls, Hs = (samp, other) if keep_low else (other, samp)
    # first sample j with P(j*stride) false (vectorised on the device, one host read)
    j = _first_false(ops.order(Ls) <= ops.order(Hs))
    lo = 0 if j == 0 else (j - 1) * stride + 1  # P(lo-1) true (or lo = 0)
    hi = m if j == Ls.numel() else j * stride   # P(hi) false (or hi = m)
    # window: L[lo:hi] and H[m-1-(hi-1) : m-1-lo+1] = H[m-hi : m-lo]
    if hi > lo:
        if keep_low:
            win = mine[lo:hi].contiguous()
        else:
            win = mine[m - hi:m - lo].contiguous()
        owin = torch.empty_like(win)
        comm.exchange(win, owin, partner)
        Lw, Hw = (win, owin) if keep_low else (owin, win)
        # P(i) = L[i] <= H[m-1-i], i in [lo, hi): L[i] = Lw[i-lo], H[m-1-i] = Hw[hi-1-i]
        c = lo + _first_false(ops.order(Lw) <= ops.order(Hw.flip(0)))
    else:
        c = lo
    return m - c


def _first_false(p: torch.Tensor) -> int:
    """Index of the first False of a true-then-false predicate vector (len if none)."""
    if p.numel() == 0:
        return 0
    return int((~p).to(torch.int32).argmax().item()) if not bool(p.all()) else p.numel()


def _on_stream(ops):
    """Run the schedule's torch work on the stream the local operations use, so a
    caller that passes HipOps(stream=s) without entering it gets ordered work (a raw
    hipStream_t handle is wrapped as an external stream)."""
    s = getattr(ops, "stream", None)
    if s is None:
        return contextlib.nullcontext()
    if isinstance(s, int):
        s = torch.cuda.ExternalStream(s)
    return torch.cuda.stream(s)


def dist_sort(local: torch.Tensor, ops: Ops, group=None, partial: bool = True, stride: int = 4096,
              copy_input: bool = False, comm=None) -> torch.Tensor:
    """Sort the global array whose rank-r shard is `local` (equal shard sizes).
    Returns this rank's shard of the sorted array (global ranks r*m .. r*m+m-1).
    `local` is sorted in place unless copy_input (then it is left untouched)."""
    with _on_stream(ops):
        return _dist_sort(local, ops, group, partial, stride, copy_input, comm)


def _dist_sort(local, ops, group, partial, stride, copy_input, comm):
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    comm = comm if comm is not None else P2PComm(group)
    if world & (world - 1):
        raise ValueError("dist_sort: world size must be a power of two")
    a = ops.local_sort(local, out_of_place=copy_input)
    m = a.numel()
    for stage, step in schedule(world):
        partner, keep_low = partner_and_side(rank, stage, step)
        if not partial:
            b = torch.empty_like(a)
            comm.exchange(a.contiguous(), b, partner)
            lo_blk, hi_blk = (a, b) if rank < partner else (b, a)  # same merge order on both sides
            a = ops.merge(lo_blk, hi_blk, 0, m) if keep_low else ops.merge(lo_blk, hi_blk, m, 2 * m)
            continue
        k = _split_count(ops, a, partner, keep_low, stride, comm)
        if k == 0:
            continue
        if keep_low:
            give = a[m - k:].contiguous()   # my top k go up
        else:
            give = a[:k].contiguous()       # my bottom k go down
        got = torch.empty_like(give)
        comm.exchange(give, got, partner)
        if keep_low:
            a = ops.merge(a[:m - k], got, 0, m)   # keep my bottom m-k + partner's bottom k
        else:
            a = ops.merge(got, a[k:], 0, m)       # partner's top k + my top m-k
    return a


class GlooColl:
    """Host collectives over a torch.distributed group (gloo): the labsort_host_coll
    callbacks of a host-staged labsort communicator (DistComm.host).  The CPU tests use
    it with the oracle's host instantiation of the schedule, the GPU tests to run several
    ranks of the HIP schedule on one GPU."""

    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group)

    def allgather(self, h_in: int, h_out: int, nbytes: int) -> None:
        import ctypes
        t = torch.empty(nbytes, dtype=torch.uint8)
        ctypes.memmove(t.data_ptr(), h_in, nbytes)
        outs = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(self.world)]
        dist.all_gather(outs, t, group=self.group)
        for i, o in enumerate(outs):
            ctypes.memmove(h_out + i * nbytes, o.data_ptr(), nbytes)

    def alltoallv(self, h_send: int, send_bytes: list, h_recv: int, recv_bytes: list) -> None:
        import ctypes
        ts, tr = sum(send_bytes), sum(recv_bytes)
        inp = torch.empty(ts // 4, dtype=torch.int32)
        if ts:
            ctypes.memmove(inp.data_ptr(), h_send, ts)
        out = torch.empty(tr // 4, dtype=torch.int32)
        dist.all_to_all_single(out, inp, [b // 4 for b in recv_bytes], [b // 4 for b in send_bytes],
                               group=self.group)
        if tr:
            ctypes.memmove(h_recv, out.data_ptr(), tr)


def make_comm(ls, backend: str = "nccl", group=None):
    """This rank's labsort communicator: RCCL (backend "nccl": rank 0's ncclUniqueId
    broadcast over the torch.distributed group) or host-staged gloo collectives."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if backend != "nccl":
        return ls.DistComm.host(world, rank, GlooColl(group))
    uid = ls.DistComm.unique_id() if rank == 0 else bytes(128)
    obj = [uid]
    dist.broadcast_object_list(obj, src=0, group=group)
    return ls.DistComm.rccl(world, rank, obj[0])


def dist_sort_splitters(local: torch.Tensor, comm, key: str = "u32", stream=None, copy: bool = True):
    """Sort the global array whose rank-r shard is `local` (device tensor, left
    untouched) with the product's splitter exchange: labsort_dist_sort, the C++ schedule
    of csrc/dist_plan.h (local radix sort, (key, rank, position) splitters from a regular
    sample, pairwise send/recv with every peer at once, merge of the received runs in
    rank order).  Returns (this rank's contiguous range of the sorted array, its global
    offset); copy=False: the range as a view of the communicator's buffer (kept alive by
    the view, invalid after the communicator's next sort: see DistComm.sort_tensor)."""
    return comm.sort_tensor(local, local.numel(), key=key, stream=stream, copy=copy)
