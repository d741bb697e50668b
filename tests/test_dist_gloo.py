"""Multi-rank tests of the merge-split exchange (dist.py) on CPU with the gloo
backend.  The local operations are injected (`NumpyOps`: numpy sort and a
stable two-run merge, A before B on ties, as lab.cu:163-170) so the schedule,
the split-count protocol and the send/recv pairing are exercised without GPUs;
on the GPU box the same schedule runs with HipOps (liblabsort) over RCCL.
The result is compared with the oracle's std::sort of the whole array."""
import importlib
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

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
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as O
        D = importlib.import_module(PKG_NAME + ".dist")

        class NumpyOps(D.Ops):
            def __init__(self, key):
                self.key = key
                self.f = np.uint32(0x80000000 if key == "i32" else 0)

            def upper_bound(self, a, values):
                av = self._u(a)
                vv = self._u(values)
                return torch.from_numpy(np.searchsorted(av, vv, side="right").astype(np.int64))

            def _u(self, t):
                return t.numpy().view(np.uint32) ^ self.f

            def local_sort(self, t, out_of_place=False):
                s = torch.from_numpy(((np.sort(self._u(t)) ^ self.f).view(np.int32)).copy())
                if out_of_place:
                    return s
                t.copy_(s)
                return t

            def merge(self, a, b, d0, d1):
                cat = np.concatenate([self._u(a), self._u(b)])
                idx = np.argsort(cat, kind="stable")  # a's elements first on ties
                return torch.from_numpy(((cat[idx][d0:d1] ^ self.f).view(np.int32)).copy())

            def key_le(self, x, y):
                f = int(self.f)
                return ((x & 0xFFFFFFFF) ^ f) <= ((y & 0xFFFFFFFF) ^ f)

        m, dist_name, seed, key = cfg["m"], cfg["dist"], cfg["seed"], cfg["key"]
        shard = O.gen(m, seed, dist_name, first=rank * m)
        t = torch.from_numpy(shard.view(np.int32).copy())
        if cfg.get("exchange") == "splitters":
            out = D.dist_sort_splitters(t, NumpyOps(key), copy_input=cfg.get("copy", False),
                                        oversample=cfg.get("oversample", 64))
        else:
            out = D.dist_sort(t, NumpyOps(key), partial=cfg["partial"], stride=cfg["stride"],
                              copy_input=cfg.get("copy", False))
        if cfg.get("copy", False):
            assert torch.equal(t, torch.from_numpy(shard.view(np.int32)))  # input untouched
        q.put((rank, out.numpy().copy()))
    finally:
        dist.destroy_process_group()


def run(world, cfg):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cfg, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    if cfg.get("max_share"):
        sizes = [res[r].size for r in range(world)]
        assert max(sizes) <= cfg["max_share"] * cfg["m"], sizes
    return np.concatenate([res[r] for r in range(world)])


CFGS = [
    dict(m=5000, dist="u32", seed=0x5EED0005, key="u32", partial=True, stride=64),
    dict(m=5000, dist="mod100", seed=0x5EED0005, key="u32", partial=True, stride=64),
    dict(m=4096, dist="u32", seed=0x5EED0006, key="i32", partial=True, stride=1000, copy=True),
    dict(m=3000, dist="mod1000", seed=0x5EED0007, key="u32", partial=False, stride=64),
    dict(m=2000, dist="const", seed=1, key="u32", partial=True, stride=7),
    dict(m=2000, dist="reversed", seed=1, key="u32", partial=True, stride=128),
    dict(m=5000, dist="u32", seed=0x5EED0008, key="u32", exchange="splitters", copy=True),
    dict(m=4000, dist="mod100", seed=0x5EED0009, key="u32", exchange="splitters"),
    dict(m=3001, dist="u32", seed=0x5EED000A, key="i32", exchange="splitters", oversample=3),
    dict(m=100, dist="const", seed=3, key="u32", exchange="splitters"),
    dict(m=1, dist="u32", seed=4, key="u32", exchange="splitters"),
    # repeated keys are cut between ranks by (key, rank, position) splitters: every
    # range stays near its share (a constant input used to land on one rank)
    dict(m=4000, dist="const", seed=5, key="u32", exchange="splitters", max_share=1.05),
    dict(m=4000, dist="mod100", seed=6, key="i32", exchange="splitters", max_share=1.05),
]


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("ci", range(len(CFGS)))
def test_dist_sort_gloo(oracle, world, ci):
    cfg = CFGS[ci]
    got = run(world, cfg)
    full = oracle.gen(cfg["m"] * world, cfg["seed"], cfg["dist"])
    if cfg["dist"] == "reversed":
        full = np.concatenate([oracle.gen(cfg["m"], cfg["seed"], "reversed", first=r * cfg["m"])
                               for r in range(world)])
    exp = oracle.sort_i32(full.view(np.int32)).view(np.uint32) if cfg["key"] == "i32" else oracle.sort_u32(full)
    np.testing.assert_array_equal(got.view(np.uint32), exp)


@pytest.mark.parametrize("ci", [0, 6, 11, 12])
def test_dist_sort_gloo_world8(oracle, ci):
    """BASELINE config 5's rank count (8) on CPU: bitonic network and splitter exchange."""
    test_dist_sort_gloo(oracle, 8, ci)


def test_schedule_shape():
    D = importlib.import_module(PKG_NAME + ".dist")
    assert len(D.schedule(8)) == 6 and len(D.schedule(2)) == 1 and D.schedule(1) == []
    # every step pairs ranks symmetrically and sides agree
    for world in (2, 4, 8):
        for stage, step in D.schedule(world):
            for r in range(world):
                p, low = D.partner_and_side(r, stage, step)
                p2, low2 = D.partner_and_side(p, stage, step)
                assert p2 == r and low != low2
