"""GPU test of the multi-GPU merge-sort path (dist.py with HipOps = liblabsort.so):
2 and 4 ranks share cuda:0 and exchange through host-staged gloo (HostStagedComm),
so the local sorts and merge-split steps run in the HIP kernels exactly as they do
over RCCL on an 8-GPU node.  The concatenated shards must equal std::sort of the
whole array (the oracle)."""
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


def _worker(rank, world, port, cfg, q):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ls = importlib.import_module(PKG_NAME)
        D = importlib.import_module(PKG_NAME + ".dist")
        m = cfg["m"]
        t = torch.empty(m, dtype=torch.int32, device="cuda")
        ls.fill(t, m, cfg["seed"], cfg["dist"], first=rank * m)
        ops = D.HipOps(ls, key=cfg["key"], local_algo=cfg["algo"], kway=cfg.get("kway", True))
        if cfg.get("exchange") == "splitters":
            out = D.dist_sort_splitters(t, ops, copy_input=True, comm=D.HostStagedComm())
        else:
            out = D.dist_sort(t, ops, partial=cfg["partial"], stride=cfg["stride"], copy_input=True,
                              comm=D.HostStagedComm())
        torch.cuda.synchronize()
        q.put((rank, out.cpu().numpy().copy()))
    finally:
        dist.destroy_process_group()


def run(world, cfg):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if cfg.get("max_share"):
        sizes = [res[r].size for r in range(world)]
        assert max(sizes) <= cfg["max_share"] * cfg["m"], sizes
    return np.concatenate([res[r] for r in range(world)])


CFGS = [
    dict(m=100_000, dist="u32", seed=0x5EED0005, key="u32", algo="radix", partial=True, stride=512),
    dict(m=1 << 20, dist="u32", seed=0x5EED0005, key="u32", algo="radix", partial=True, stride=4096),
    dict(m=65_537, dist="mod100", seed=0x5EED0006, key="u32", algo="merge", partial=True, stride=1000),
    dict(m=50_000, dist="u32", seed=0x5EED0007, key="i32", algo="radix", partial=False, stride=64),
    # splitter exchange; received runs merged by the product default (one K-way
    # labsort_merge_runs pass), and one config through the labsort_merge tree
    dict(m=1 << 20, dist="u32", seed=0x5EED0008, key="u32", algo="radix", exchange="splitters"),
    dict(m=300_001, dist="mod1000", seed=0x5EED0009, key="i32", algo="radix", exchange="splitters"),
    dict(m=70_000, dist="const", seed=0x5EED000A, key="u32", algo="radix", exchange="splitters", max_share=1.02),
    dict(m=1 << 20, dist="u32", seed=0x5EED000B, key="u32", algo="radix", exchange="splitters", kway=False),
    dict(m=200_003, dist="mod100", seed=0x5EED000C, key="i32", algo="radix", exchange="splitters",
         max_share=1.02),
    dict(m=150_000, dist="sorted", seed=0x5EED000D, key="u32", algo="radix", exchange="splitters",
         max_share=1.02),
    dict(m=1, dist="u32", seed=0x5EED000E, key="u32", algo="radix", exchange="splitters"),  # tiny shards
]


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("ci", range(len(CFGS)))
def test_dist_sort_hip(oracle, world, ci):
    cfg = CFGS[ci]
    got = run(world, cfg).view(np.uint32)
    full = oracle.gen(cfg["m"] * world, cfg["seed"], cfg["dist"])
    exp = oracle.sort_i32(full.view(np.int32)).view(np.uint32) if cfg["key"] == "i32" else oracle.sort_u32(full)
    np.testing.assert_array_equal(got, exp)


@pytest.mark.parametrize("ci", [1, 4, 6, 7, 8])
def test_dist_sort_hip_world8(oracle, ci):
    """BASELINE config 5's rank count: 8 ranks (sharing cuda:0, host-staged exchange)
    through the HIP local sorts and merges, bitonic network and splitter exchange."""
    test_dist_sort_hip(oracle, 8, ci)
