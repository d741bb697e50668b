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

`dist_sort_splitters` is the all-link form (the default of bench.py): every rank
sorts its shard, the ranks agree on p-1 splitters from a regular sample of every
shard (one all_gather), cut their sorted shards at the splitters
(`labsort_upper_bound`), send piece j to rank j with pairwise send/recv posted to
all peers at once (so all 7 xGMI links of a node carry data together instead of
one per step) straight into one buffer, and merge the p received runs in rank
order in one K-way `labsort_merge_runs` pass (or a tree of `labsort_merge` passes;
A before B on ties).  Rank r then holds the r-th contiguous
range of the sorted array; range sizes follow the splitters (within a few percent
of n/p on varied data; skewed data with a heavy repeated key can unbalance them).

Local operations are pluggable (`Ops`): the product uses liblabsort.so on the
rank's GPU (`HipOps`); the CPU tests inject an oracle-backed implementation so the
exchange schedule is exercised with the gloo backend on machines without GPUs.
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

    def merge_runs(self, buf: torch.Tensor, offsets: list) -> torch.Tensor:
        """Merge of the sorted runs buf[offsets[q]:offsets[q+1]] in run order (equal
        keys keep run order).  Default: a tree of pairwise merges."""
        runs = [buf[offsets[q]:offsets[q + 1]] for q in range(len(offsets) - 1)]
        while len(runs) > 1:
            nxt = []
            for i in range(0, len(runs) - 1, 2):
                x, y = runs[i], runs[i + 1]
                if x.numel() == 0:
                    nxt.append(y)
                elif y.numel() == 0:
                    nxt.append(x)
                else:
                    nxt.append(self.merge(x, y, 0, x.numel() + y.numel()))
            if len(runs) % 2:
                nxt.append(runs[-1])
            runs = nxt
        return runs[0].contiguous() if runs else buf[:0]

    def key_le(self, x: int, y: int) -> bool:
        raise NotImplementedError

    def argsort(self, t: torch.Tensor) -> torch.Tensor:
        """Stable argsort of int32-stored keys in key order (int64 indices)."""
        return torch.argsort(self.order(t), stable=True)

    def upper_bound(self, a: torch.Tensor, values: torch.Tensor) -> torch.Tensor:
        """int64 tensor: number of keys of sorted `a` <= each value (key order)"""
        raise NotImplementedError

    def order(self, t: torch.Tensor) -> torch.Tensor:
        """int64 view of int32-stored keys that is monotone in key order"""
        f = 0x80000000 if getattr(self, "key", "u32") == "i32" else 0
        return (t.to(torch.int64) & 0xFFFFFFFF) ^ f


class HipOps(Ops):
    """liblabsort.so on the current GPU."""

    def __init__(self, ls, key: str = "u32", local_algo: str = "radix", stream=None, kway: bool = True):
        self.ls, self.key, self.algo, self.stream = ls, key, local_algo, stream
        # kway: merge the received runs with labsort_merge_runs (pair passes over explicit
        # runs in C++) instead of a Python tree of labsort_merge calls.  Measured on
        # MI355X for 2^28 keys in p runs (profiles/r17_dist_merge_step.jsonl): p = 2 / 4 /
        # 8: 0.53 / 1.04 / 1.66 ms, tree 0.75 / 1.45 / 2.22 ms
        self.kway = kway
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

    def argsort(self, t):
        """Stable argsort by the labsort key/value sort of (key, index) pairs."""
        n = t.numel()
        if n == 0:
            return torch.zeros(0, dtype=torch.int64, device=t.device)
        idx = torch.arange(n, dtype=torch.int32, device=t.device)
        ko, vo = torch.empty_like(t), torch.empty_like(idx)
        ws = torch.empty(max(self.ls.pairs_workspace_bytes(n, "auto"), 256), dtype=torch.uint8, device=t.device)
        self.ls.sort_pairs_device(t.contiguous(), idx, ko, vo, n, key=self.key, algo="auto", workspace=ws,
                                  stream=self.stream)
        self.ls.pairs_workspace_status(ws, n, "auto", stream=self.stream)
        return vo.to(torch.int64)

    def merge(self, a, b, d0, d1):
        out = torch.empty(max(d1 - d0, 1), dtype=torch.int32, device=a.device if a.numel() else b.device)
        parts = self.ls.merge_parts(d1 - d0)
        if self._part is None or self._part.numel() < parts:
            self._part = torch.empty(parts, dtype=torch.int32, device=out.device)
        self.ls.merge(a, a.numel(), b, b.numel(), out, d0, d1, self._part, key=self.key, stream=self.stream)
        return out[: d1 - d0]

    def merge_runs(self, buf, offsets):
        """One K-way pass (labsort_merge_runs, K <= 8) when self.kway (the default);
        otherwise, and for more than 8 runs, the merge tree."""
        if not self.kway or len(offsets) - 1 > 8:
            return super().merge_runs(buf, offsets)
        n = offsets[-1] - offsets[0]
        out = torch.empty(max(n, 1), dtype=torch.int32, device=buf.device)
        if n:
            o = [x - offsets[0] for x in offsets]
            self.ls.merge_runs(buf[offsets[0]:offsets[-1]], out, o, key=self.key, workspace=self._kmws(n),
                               stream=self.stream)
        return out[:n]

    def _kmws(self, n):
        need = max(self.ls.merge_runs_workspace_bytes(n), 256)
        if getattr(self, "_km", None) is None or self._km.numel() < need:
            self._km = torch.empty(need, dtype=torch.uint8, device="cuda")
        return self._km

    def key_le(self, x, y):
        f = 0x80000000 if self.key == "i32" else 0
        return ((x & 0xFFFFFFFF) ^ f) <= ((y & 0xFFFFFFFF) ^ f)

    def upper_bound(self, a, values):
        out = torch.empty(values.numel(), dtype=torch.int32, device=a.device)
        self.ls.upper_bound(a, a.numel(), values.contiguous(), values.numel(), out, key=self.key,
                            stream=self.stream)
        return out.to(torch.int64)


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

    def exchange_all(self, sends: list, recvs: list, rank: int) -> None:
        """sends[j] -> rank j, recvs[j] <- rank j for every peer j != rank, all posted
        together (one group: every xGMI link busy at once); empty pieces are skipped."""
        self.sent_bytes += sum(x.numel() * x.element_size() for j, x in enumerate(sends) if j != rank)
        self.p2p_rounds += 1
        g = self.group
        ops = []
        for j in range(len(sends)):
            if j == rank:
                continue
            if sends[j].numel():
                ops.append(dist.P2POp(dist.isend, sends[j], j, group=g))
            if recvs[j].numel():
                ops.append(dist.P2POp(dist.irecv, recvs[j], j, group=g))
        self._sync()
        t0 = time.perf_counter()
        if ops:
            for r in dist.batch_isend_irecv(ops):
                r.wait()
        self._sync()
        self.exchange_s += time.perf_counter() - t0

    def all_gather(self, t: torch.Tensor) -> list:
        out = [torch.empty_like(t) for _ in range(dist.get_world_size(self.group))]
        dist.all_gather(out, t, group=self.group)
        return out


class HostStagedComm(P2PComm):
    """Test adapter: device tensors are staged through host memory and exchanged
    with a CPU backend (gloo), so the GPU-side schedule (HipOps on one device) can
    be exercised by several processes sharing one GPU."""

    def exchange(self, send, recv, partner):
        hs = send.cpu()
        hr = torch.empty_like(hs)
        super().exchange(hs, hr, partner)
        recv.copy_(hr)

    def exchange_all(self, sends, recvs, rank):
        hs = [x.cpu() if j != rank else x[:0].cpu() for j, x in enumerate(sends)]
        hr = [torch.empty(x.shape, dtype=x.dtype) if j != rank else x[:0].cpu() for j, x in enumerate(recvs)]
        super().exchange_all(hs, hr, rank)
        for j, (d, h) in enumerate(zip(recvs, hr)):
            if j != rank and h.numel():
                d.copy_(h)

    def all_gather(self, t):
        return [x.to(t.device) for x in super().all_gather(t.cpu())]


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
    caller that passes HipOps(stream=s) without entering it gets ordered work."""
    s = getattr(ops, "stream", None)
    return torch.cuda.stream(s) if s is not None else contextlib.nullcontext()


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


def dist_sort_splitters(local: torch.Tensor, ops: Ops, group=None, comm=None, copy_input: bool = False,
                        oversample: int = 1024) -> torch.Tensor:
    """Sort the global array whose rank-r shard is `local` with one all-peer exchange.
    Returns this rank's contiguous range of the sorted array (ranges in rank order).

    Splitters are (key, source rank, position) triples, so runs of one repeated key
    are cut between ranks like any other keys: every range stays within the sample
    granularity (about n/oversample keys) of its share, even for constant input."""
    with _on_stream(ops):
        return _dist_sort_splitters(local, ops, group, comm, copy_input, oversample)


def _dist_sort_splitters(local, ops, group, comm, copy_input, oversample):
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    comm = comm if comm is not None else P2PComm(group)
    a = ops.local_sort(local, out_of_place=copy_input)
    if world == 1:
        return a
    m = a.numel()
    # regular sample of every sorted shard: (key, position); the same sample size on
    # every rank (all_gather), positions repeat if m < s
    s = oversample * world
    idx = (torch.arange(s, device=a.device, dtype=torch.int64) * m) // s
    samp = a[idx].contiguous() if m else torch.zeros(s, dtype=a.dtype, device=a.device)
    meta = torch.cat([idx, torch.tensor([1 if m else 0], dtype=torch.int64, device=a.device)])
    samples = comm.all_gather(samp)
    metas = comm.all_gather(meta)
    valid = [int(x) for x in torch.stack([mt[-1] for mt in metas]).cpu().tolist()]  # empty shards sample nothing
    ranks_ok = [r for r in range(world) if valid[r]]
    if not ranks_ok:
        ranks_ok = [rank]
    pool = torch.cat([samples[r] for r in ranks_ok])
    pool_rank = torch.cat([torch.full((s,), r, dtype=torch.int64, device=a.device) for r in ranks_ok])
    pool_pos = torch.cat([metas[r][:-1] for r in ranks_ok])
    # rank order + ascending positions per rank + a stable sort by key = (key, rank, pos) order
    srt = ops.argsort(pool)
    q = srt[(torch.arange(1, world, device=a.device, dtype=torch.int64) * pool.numel()) // world]
    spl_key, spl_rank, spl_pos = pool[q].contiguous(), pool_rank[q], pool_pos[q]
    # cut j on this rank: keys before splitter j in (key, rank, pos) order
    if m:
        f = 0x80000000 if getattr(ops, "key", "u32") == "i32" else 0
        o = ops.order(spl_key)
        prev = ((o - 1).clamp(min=0) ^ f) & 0xFFFFFFFF            # key just below, in key order
        prev = torch.where(prev >= 2**31, prev - 2**32, prev).to(torch.int32)
        both = ops.upper_bound(a, torch.cat([spl_key, prev]))
        ub, lb = both[:world - 1], torch.where(o == 0, torch.zeros_like(o), both[world - 1:])
        cuts = torch.where(spl_rank > rank, ub, torch.where(spl_rank < rank, lb, spl_pos + 1))
    else:
        cuts = torch.zeros(world - 1, dtype=torch.int64, device=a.device)
    bounds = [0] + [int(c) for c in cuts.cpu().tolist()] + [m]
    sizes = torch.tensor([bounds[j + 1] - bounds[j] for j in range(world)], dtype=torch.int64, device=a.device)
    all_sizes = torch.stack(comm.all_gather(sizes)).cpu()  # all_sizes[i][j] = rank i -> rank j
    sends = [a[bounds[j]:bounds[j + 1]] for j in range(world)]
    # receive every piece straight into its slot of one buffer (rank order), then merge
    # the p runs (A before B on ties, so equal keys keep rank order)
    counts = [int(all_sizes[i][rank]) for i in range(world)]
    offs = [0]
    for c in counts:
        offs.append(offs[-1] + c)
    buf = torch.empty(max(offs[-1], 1), dtype=a.dtype, device=a.device)
    recvs = [buf[offs[i]:offs[i + 1]] for i in range(world)]
    if counts[rank]:
        recvs[rank].copy_(sends[rank])
    comm.exchange_all([x.contiguous() for x in sends], recvs, rank)
    return ops.merge_runs(buf, offs)
