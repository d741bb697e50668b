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


# ---- a failing rank ends every rank (the status words of dist_plan.h's collectives) ----
FAIL_CASES = [("local_sort", 1), ("bounds", 0), ("recv", -1), ("grow", 1)]


def _skewed(ls, torch, rank, m):
    """rank 0: m keys below 2^31; rank r > 0: 1000 keys above every key of the ranks
    before it -- range 0 outgrows the pre-sized receive buffer (the growth round)"""
    if rank == 0:
        t = torch.empty(m, dtype=torch.int32, device="cuda")
        ls.fill(t, m, 0x5EED0015, "u31")
        return t
    t = torch.empty(1000, dtype=torch.int32, device="cuda")
    ls.fill(t, 1000, 0x5EED0015, "u32", first=rank * 1000)
    return (t & 0x00FFFFFF) | ((0x80000000 + (rank << 24)) - (1 << 32))  # (the int32 of that word)


def _fail_worker(rank, world, port, q):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import time

    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ls = importlib.import_module(PKG_NAME)
        D = importlib.import_module(PKG_NAME + ".dist")
        comm = D.make_comm(ls, backend="gloo")
        m = 200_000
        t = torch.empty(m, dtype=torch.int32, device="cuda")
        ls.fill(t, m, 0x5EED0012, "u32", first=rank * m)
        skew = _skewed(ls, torch, rank, m)
        for ci, (phase, fr) in enumerate(FAIL_CASES):
            ls.test_fault(phase, fr % world)
            x = skew if phase == "grow" else t
            t0 = time.monotonic()
            try:
                comm.sort(x, x.numel())
                st = 0
            except ls.LabsortError as e:
                st = e.status
            q.put((ci, rank, st, time.monotonic() - t0))
        ls.test_fault(None)
        out, goff = D.dist_sort_splitters(skew, comm)  # the growth round, then the sorted ranges
        torch.cuda.synchronize()
        q.put((len(FAIL_CASES) + 1, rank, 0, (out.cpu().numpy().copy(), goff)))
        out, goff = D.dist_sort_splitters(t, comm)  # the communicator still works
        torch.cuda.synchronize()
        q.put((len(FAIL_CASES), rank, 0, (out.cpu().numpy().copy(), goff)))
        comm.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_dist_sort_failure_ends_every_rank(oracle, world):
    """labsort_dist_sort with one rank's local sort, bound queries, receive buffer or
    buffer growth failing (ls.test_fault): that rank returns LABSORT_ERR_DEVICE, every
    other rank LABSORT_ERR_PEER, each within seconds, and the next sorts on the same
    communicators succeed (one of them on skewed shards, through the growth round)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_fail_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world * (len(FAIL_CASES) + 2)):
        ci, r, st, extra = q.get(timeout=300)
        got[(ci, r)] = (st, extra)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for ci, (phase, fr) in enumerate(FAIL_CASES):
        for r in range(world):
            st, secs = got[(ci, r)]
            assert st == (3 if r == fr % world else 4), (phase, r, st)
            assert secs < 30, (phase, r, secs)
    m = 200_000
    exp = oracle.sort_u32(oracle.gen(m * world, 0x5EED0012, "u32"))
    np.testing.assert_array_equal(np.concatenate([got[(len(FAIL_CASES), r)][1][0] for r in range(world)]).view(np.uint32),
                                  exp)
    # skewed shards: range 0 = all of shard 0, through the growth round
    skew = [oracle.gen(m, 0x5EED0015, "u31")] + [
        (oracle.gen(1000, 0x5EED0015, "u32", first=r * 1000) & np.uint32(0x00FFFFFF)) | np.uint32(0x80000000 + (r << 24))
        for r in range(1, world)]
    parts = [got[(len(FAIL_CASES) + 1, r)][1] for r in range(world)]
    # range 0: all of shard 0 (+ the splitter key itself), past the pre-sized buffer
    assert parts[0][0].size >= m and [g for _, g in parts] == list(np.cumsum([0] + [o.size for o, _ in parts])[:-1])
    np.testing.assert_array_equal(np.concatenate([o for o, _ in parts]).view(np.uint32),
                                  oracle.sort_u32(np.concatenate(skew)))


def _exchange_fail_worker(rank, world, port, q):
    """rank 1 leaves at the exchange without taking part (ls.test_fault("exchange", 1)):
    the peers' host-staged all-to-all must end (gloo timeout 10 s, or the failed rank's
    connections closing); the group is unusable afterwards, so the process just ends"""
    import datetime
    import time
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=10))
    ls = importlib.import_module(PKG_NAME)
    D = importlib.import_module(PKG_NAME + ".dist")
    comm = D.make_comm(ls, backend="gloo")
    m = 100_000
    t = torch.empty(m, dtype=torch.int32, device="cuda")
    ls.fill(t, m, 0x5EED0016, "u32", first=rank * m)
    ls.test_fault("exchange", 1)
    t0 = time.monotonic()
    try:
        comm.sort(t, m)
        st = 0
    except ls.LabsortError as e:
        st = e.status
    torch.cuda.synchronize()
    q.put((rank, st, time.monotonic() - t0))
    q.close()
    q.join_thread()
    os._exit(0)


@pytest.mark.parametrize("world", [2, 4])
def test_dist_sort_exchange_failure_ends_every_rank(world):
    """VERDICT r4 item 3 on the HIP instantiation (host-staged communicator over gloo): one
    rank fails inside the exchange; it returns LABSORT_ERR_DEVICE, every other rank
    LABSORT_ERR_PEER, all within 30 s."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_exchange_fail_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        r, st, secs = q.get(timeout=180)
        got[r] = (st, secs)
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        st, secs = got[r]
        assert st == (3 if r == 1 else 4), (r, st)
        assert secs < 30, (r, secs)


def _rccl_init_alone(q):
    """rank 0 of a 2-rank RCCL communicator whose rank 1 never joins: the nonblocking
    ncclCommInitRankConfig must end at the communicator deadline (3 s here) with
    LABSORT_ERR_PEER, not block forever"""
    import time
    sys.path.insert(0, REPO)
    import torch
    torch.cuda.set_device(0)
    ls = importlib.import_module(PKG_NAME)
    ls.set_comm_timeout(3.0)
    uid = ls.DistComm.unique_id()
    t0 = time.monotonic()
    try:
        ls.DistComm.rccl(2, 0, uid)
        st = 0
    except ls.LabsortError as e:
        st = e.status
    q.put((st, time.monotonic() - t0))
    q.close()
    q.join_thread()
    os._exit(0)


def test_rccl_init_peer_never_joins():
    """RCCL communicator creation is bounded: a peer that never joins ends the wait at the
    deadline (LABSORT_ERR_PEER) and the half-made communicator is aborted."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_init_alone, args=(q,))
    p.start()
    st, secs = q.get(timeout=120)
    p.join(timeout=60)
    assert st == 4, st
    assert 2.5 < secs < 30, secs


def test_bench_dist_gloo_config5():
    """bench.py's N > 1 line rehearsed with 2 ranks on one GPU over gloo: BASELINE config 5
    (2^30 keys partitioned over the ranks: 2^29 each, strong scaling), verified."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
                        os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "gloo", "--steps", "1",
                        "--warmup", "0", "--no-weak", "--no-host-path"],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert "BASELINE config 5" in line["config"]["workload"]
    assert line["config"]["n_total"] == 1 << 30 and line["config"]["n_per_gpu"] == 1 << 29
    ph = line["xgmi"]["phases_ms_last_step"]
    assert ph["plan_work"] >= 0 and ph["plan_wait"] >= 0
    assert set(line["xgmi"]["collectives_ms_last_step"]) >= {"samples", "counts"}


def test_bench_plain_gpus2_launches_ranks():
    """`python3 bench.py --gpus 2` WITHOUT torch.distributed.run (how the driver invokes the
    bench): bench.py starts the two ranks itself and relays rank 0's config-5 line"""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--steps", "1", "--warmup", "0", "--no-weak", "--no-host-path", "--total-log2n", "26"],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert "BASELINE config 5" in line["config"]["workload"]
    assert line["config"]["n_total"] == 1 << 26 and line["value"] > 0


def test_bench_plain_gpus8_nccl_refused_on_one_gpu():
    """--gpus 8 over RCCL on a box with fewer GPUs: refused at once, non-zero"""
    import subprocess
    import time
    import torch
    if torch.cuda.device_count() >= 8:
        pytest.skip("an 8-GPU box runs the real thing")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "8", "--steps", "1"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0
    assert time.monotonic() - t0 < 30
    assert "needs 8 GPUs" in r.stderr
