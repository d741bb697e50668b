"""GPU tests of the one-process-per-GPU merge-sort path: 2, 4 and 8 processes share
cuda:0.
* Splitter exchange = the product: labsort_dist_sort (csrc/dist_plan.h's schedule on
  the HIP rank operations) over a host-staged communicator whose collectives are
  torch.distributed gloo (DistComm.host + dist.GlooColl) -- the same C++ code bench.py
  --gpus N runs over RCCL (DistComm.rccl), which is exercised here with one rank.
* Bitonic merge-split network (dist.dist_sort with HipOps), host-staged.
The concatenated ranges must equal std::sort of the whole array (the oracle)."""
import importlib
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_NAME = "radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd"


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_cfg(ls, D, torch, rank, world, cfg):
    m = cfg["m"]
    t = torch.empty(m, dtype=torch.int32, device="cuda")
    ls.fill(t, m, cfg["seed"], cfg["dist"], first=rank * m)
    if cfg.get("exchange") == "splitters":
        comm = D.make_comm(ls, backend="gloo")
        src = t.clone()
        out, goff = D.dist_sort_splitters(t, comm, key=cfg["key"])
        torch.cuda.synchronize()
        assert torch.equal(t, src)  # the shard is left untouched
        ph, sent = comm.timing()
        assert ph["local_sort"] > 0 and sent <= 4 * m
        res = (out.cpu().numpy().copy(), goff)
        comm.close()
        return res
    ops = D.HipOps(ls, key=cfg["key"], local_algo=cfg["algo"])
    out = D.dist_sort(t, ops, partial=cfg["partial"], stride=cfg["stride"], copy_input=True,
                      comm=D.HostStagedComm())
    torch.cuda.synchronize()
    return out.cpu().numpy().copy(), None


def _worker(rank, world, port, cfgs, q):
    """one rank: every config in turn over one gloo group"""
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ls = importlib.import_module(PKG_NAME)
        D = importlib.import_module(PKG_NAME + ".dist")
        for ci, cfg in cfgs:
            q.put((ci, rank, _run_cfg(ls, D, torch, rank, world, cfg)))
    finally:
        dist.destroy_process_group()


def run_all(world, cfgs):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfgs, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world * len(cfgs)):
        ci, r, res = q.get(timeout=300)
        got[(ci, r)] = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out = {}
    for ci, cfg in cfgs:
        res = {r: got[(ci, r)][0] for r in range(world)}
        if got[(ci, 0)][1] is not None:  # splitter exchange: ranges at their global offsets
            off = 0
            for r in range(world):
                assert got[(ci, r)][1] == off, (ci, r)
                off += res[r].size
        if cfg.get("max_share"):
            sizes = [res[r].size for r in range(world)]
            assert max(sizes) <= cfg["max_share"] * cfg["m"], (ci, sizes)
        out[ci] = np.concatenate([res[r] for r in range(world)])
    return out


CFGS = [
    dict(m=100_000, dist="u32", seed=0x5EED0005, key="u32", algo="radix", partial=True, stride=512),
    dict(m=1 << 20, dist="u32", seed=0x5EED0005, key="u32", algo="radix", partial=True, stride=4096),
    dict(m=65_537, dist="mod100", seed=0x5EED0006, key="u32", algo="merge", partial=True, stride=1000),
    dict(m=50_000, dist="u32", seed=0x5EED0007, key="i32", algo="radix", partial=False, stride=64),
    # splitter exchange: the product (labsort_dist_sort)
    dict(m=1 << 20, dist="u32", seed=0x5EED0008, key="u32", algo="radix", exchange="splitters"),
    dict(m=300_001, dist="mod1000", seed=0x5EED0009, key="i32", algo="radix", exchange="splitters"),
    dict(m=70_000, dist="const", seed=0x5EED000A, key="u32", algo="radix", exchange="splitters", max_share=1.02),
    dict(m=(1 << 20) + 3, dist="u32", seed=0x5EED000B, key="u32", algo="radix", exchange="splitters"),
    dict(m=200_003, dist="mod100", seed=0x5EED000C, key="i32", algo="radix", exchange="splitters",
         max_share=1.02),
    dict(m=150_000, dist="sorted", seed=0x5EED000D, key="u32", algo="radix", exchange="splitters",
         max_share=1.02),
    dict(m=1, dist="u32", seed=0x5EED000E, key="u32", algo="radix", exchange="splitters"),  # tiny shards
]


def _check_world(oracle, world, indices):
    cfgs = [(ci, CFGS[ci]) for ci in indices]
    got = run_all(world, cfgs)
    for ci, cfg in cfgs:
        full = oracle.gen(cfg["m"] * world, cfg["seed"], cfg["dist"])
        exp = oracle.sort_i32(full.view(np.int32)).view(np.uint32) if cfg["key"] == "i32" else oracle.sort_u32(full)
        np.testing.assert_array_equal(got[ci].view(np.uint32), exp, err_msg=f"config {ci}")


@pytest.mark.parametrize("world", [2, 4])
def test_dist_sort_hip(oracle, world):
    """every config: bitonic network (0-3) and the product's splitter exchange (4-10)"""
    _check_world(oracle, world, range(len(CFGS)))


def test_dist_sort_hip_world8(oracle):
    """BASELINE config 5's rank count: 8 ranks (sharing cuda:0, host-staged exchange)
    through the HIP local sorts and merges, bitonic network and splitter exchange."""
    _check_world(oracle, 8, [1, 4, 6, 7, 8, 10])


def test_dist_sort_rccl_one_rank(ls, oracle, torch_gpu):
    """The RCCL communicator of bench.py --gpus N (ncclGetUniqueId, ncclCommInitRank,
    ncclAllGather, grouped send/recv) with one rank: the whole schedule on cuda:0."""
    torch = torch_gpu
    comm = ls.DistComm.rccl(1, 0, ls.DistComm.unique_id())
    try:
        for n, dist, key in [((1 << 22) + 5, "u32", "u32"), (100_003, "mod1000", "i32"), (0, "u32", "u32")]:
            t = torch.empty(max(n, 1), dtype=torch.int32, device="cuda")
            ls.fill(t, n, 0x5EED7600 + n, dist)
            out, goff = comm.sort_tensor(t, n, key=key)
            torch.cuda.synchronize()
            a = oracle.gen(n, 0x5EED7600 + n, dist)
            exp = oracle.sort_i32(a.view(np.int32)).view(np.uint32) if key == "i32" else oracle.sort_u32(a)
            assert goff == 0 and out.numel() == n
            np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), exp)
    finally:
        comm.close()
