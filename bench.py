"""bench.py -- BASELINE.json's headline metric: Mkeys/s sorting uint32 keys.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--algo radix|merge] [--log2n 28]

N = 1: one "step" is one device-resident sort of n = 2^28 uniform uint32 keys
(BASELINE config 3: radix, 1 MI355X) through liblabsort's C-ABI
(`labsort_sort_device`, the stages of order_array between its H2D and D2H
copies, lab.cu:321-397).  Keys are generated on the device (counter-based
generator, seed 0x5EED0003) and stay resident in HBM; the sort is out of place
so every step sorts the same input.

N > 1 (one process per GPU, RCCL; started by torch.distributed.run, or -- when bench.py is
invoked plainly with --gpus N -- by bench.py itself, which then launches the N ranks as one
torch.distributed.run child tree with a deadline and relays rank 0's line): BASELINE config 5,
the merge-sort path of the north_star through the product's C-ABI: a 2^30-key array
(--total-log2n) partitioned over the N ranks (2^30/N keys each: strong scaling); every
rank calls labsort_dist_sort on its communicator (labsort_comm_init_rccl, rank 0's unique
id broadcast over torch.distributed), which sorts its shard locally with the radix
kernels, moves keys by grouped ncclSend/ncclRecv at the splitters and merges its received
runs (csrc/dist_plan.h).  value = all ranks' keys / max-over-ranks time.  The same
schedule with 2^log2n keys per rank (weak scaling) is reported beside it ("weak").
--exchange pairwise runs the Python bitonic merge-split network (dist.py) instead;
--backend gloo runs the schedule over host collectives (several ranks on one GPU: a
rehearsal, not a measurement of xGMI).

host_path (after the timed region, rank 0, in a child process): the reference's
own calling convention -- a pageable host int* of 2^30 keys (BASELINE config 5)
sorted in place, PCIe copies included: labsort_sort_host on one GPU, and at N > 1
labsort_sort_host_multi over devices 0..N-1 (per-GPU PCIe shards + RCCL exchange).
Reported beside the headline, never as `value`.

After the timed region the output is verified with size-independent properties
(no descents, same sum / sum of squares / digit histograms as the input);
a failed check aborts the bench.  The printed JSON line carries:
  roofline     the dominant kernel (radix: the onesweep scatter pass) -- achieved
               = algorithmic bytes per launch (8 B/key: read + write each key once)
               / average launch duration from HIP events recorded on the sort's
               stream during the timed region; traffic = HBM bytes per launch from
               the committed rocprofv3 PMC pass (profiles/), or null.
  cpu_baseline std::sort (the oracle: oracle/cpu_sort.cpp) on one host core over a
               bounded sample of the same workload (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import glob
import importlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_NAME = "radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SEED = 0x5EED0000


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--algo", default="radix", choices=["radix", "merge", "radix1", "pairs"],
                    help="pairs: stable key/value sort (sort_by_key) of (key, uint32 index) pairs")
    ap.add_argument("--pair-algo", default="radix", choices=["radix", "merge"], help="--algo pairs: which path")
    ap.add_argument("--log2n", type=int, default=28, help="N = 1: keys = 2^log2n; N > 1: keys per GPU of the weak-scaling field")
    ap.add_argument("--total-log2n", type=int, default=30,
                    help="N > 1: the whole array (BASELINE config 5: 2^30 keys) partitioned over the N ranks")
    ap.add_argument("--no-weak", action="store_true", help="N > 1: skip the weak-scaling (2^log2n per GPU) field")
    ap.add_argument("--dist", default="u32")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-merge", action="store_true", help="skip the merge-sort leg (config 4) of the N=1 radix run")
    ap.add_argument("--cpu-seconds", type=float, default=16.0, help="budget of the CPU baseline samples")
    ap.add_argument("--exchange", default="splitters", choices=["splitters", "pairwise"],
                    help="N>1: all-peer splitter exchange + merge tree, or the bitonic pairwise merge-split network")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="N>1 only; gloo (+ host-staged exchange) is a test mode for several ranks on one GPU")
    ap.add_argument("--no-host-path", action="store_true", help="skip the host-pointer (PCIe-inclusive) leg")
    ap.add_argument("--host-log2n", type=int, default=30, help="host-pointer leg: keys = 2^host-log2n")
    ap.add_argument("--host-leg", default="", help=argparse.SUPPRESS)  # child of host_path: "peer" or "rccl"
    ap.add_argument("--launch-timeout", type=float, default=900.0,
                    help="N>1 started without torch.distributed.run: deadline for the N child ranks (s)")
    return ap.parse_args()


def pmc_traffic(kernel_class: str, n: int):
    """HBM bytes per launch of the dominant kernel from the newest committed PMC
    summary (profiles/*_pmc.json, written by profiles/pmc_summary.py from separate
    rocprofv3 --pmc passes, FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM).
    Only used when the summary was taken on the same n."""
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc.json")))
    for f in reversed(files):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        k = d.get("kernels", {}).get(kernel_class)
        if k and int(d.get("n", -1)) == n and k.get("hbm_bytes_per_launch"):
            how = (f"read x{k['read_factor']} ({k['read_shape']}), write x{k['write_factor']} ({k['write_shape']}) "
                   "from the pmc_cal calibration" if d.get("calibration") and "read_factor" in k
                   else "read x2 (guide, 16-B reads), write as measured (uncalibrated)")
            return float(k["hbm_bytes_per_launch"]), os.path.relpath(f, REPO) + ": " + how
    return None, None


def verify(torch, ls, src, out, n, key):
    """Size-independent checks: out is sorted and a permutation of src (multiset
    fingerprints: sum, sum of squares mod 2^64, 8-bit digit histograms)."""
    cnt = torch.zeros(1, dtype=torch.int32, device=out.device)
    ls.count_descents(out, n, cnt, key=key)
    hs = torch.zeros(4 * 256, dtype=torch.int32, device=out.device)
    ho = torch.zeros(4 * 256, dtype=torch.int32, device=out.device)
    ls.histogram(src, n, hs, bits=8, key=key)
    ls.histogram(out, n, ho, bits=8, key=key)

    def fp(t):
        v = t.to(torch.int64) & 0xFFFFFFFF
        s1 = int(v.sum().item())
        s2 = int((v * v).sum().item())  # wraps mod 2^64: a fingerprint, not a value
        return s1, s2

    ok = int(cnt.item()) == 0 and torch.equal(hs, ho) and fp(src) == fp(out)
    return ok, int(cnt.item())


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads() -> int:
    """Host threads this process may use: its CPU affinity, capped by OMP_NUM_THREADS
    (the GPU box gives one GPU's job a 16-thread share of a larger machine)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    return max(1, min(aff, int(omp))) if omp and omp.isdigit() else aff


def cpu_baseline(budget_s: float, n: int, ls):
    """CPU sorts of the same workload (uniform uint32 keys from the same generator,
    seed 0x5EED0003) on the host cores of the GPU box, as SURVEY §8(d) lists them:
      std::sort            1 core, 2^24-key samples repeated for ~budget_s/2 (the headline)
      __gnu_parallel::sort all usable threads, the full n, 2 repetitions
      thrust::sort (host)  the reference's "Trust" column (lab.cu:404-406): rocThrust's
                           sequential host radix sort on an int* buffer, 1 core, 2^24 samples
    All Mkeys/s.  `value` is std::sort: the oracle (kind "port")."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O  # test infrastructure: the CPU baseline leg only

    ns = 1 << 24
    keys = O.gen(ns, SEED + 3, "u32")
    t, reps = 0.0, 0
    while t < budget_s / 2 and reps < 64:
        t += O.time_sort_u32(keys, threads=1, reps=1)
        reps += 1
    thr = cpu_threads()
    full = O.gen(n, SEED + 3, "u32")
    tp = O.time_sort_u32(full, threads=thr, reps=2) / 2
    del full
    tt, treps = 0.0, 0
    while tt < budget_s / 4 and treps < 64:
        buf = keys.view(np.int32).copy()
        t0 = time.perf_counter()
        ls.order_with_trust(buf)
        tt += time.perf_counter() - t0
        treps += 1
    return {"value": round(ns * reps / t / 1e6, 2), "unit": "Mkeys/s", "cores": 1, "kind": "port",
            "sample": f"std::sort of {reps} x 2^24 uniform uint32 keys (same generator, seed 0x5EED0003), "
                      f"{t:.1f} s on one host core",
            "nproc": os.cpu_count(), "cpu_model": cpu_model(),
            "parallel": {"value": round(n / tp / 1e6, 2), "unit": "Mkeys/s", "cores": thr,
                         "sample": f"__gnu_parallel::sort of the full 2^{n.bit_length() - 1} keys, "
                                   f"{thr} threads, mean of 2 ({tp:.2f} s each)"},
            "thrust_host": {"value": round(ns * treps / tt / 1e6, 2), "unit": "Mkeys/s", "cores": 1,
                            "sample": f"rocThrust thrust::sort on a host int* (order_with_trust, lab.cu:404), "
                                      f"{treps} x 2^24 keys, {tt:.1f} s"}}


def _config1_fixture():
    return json.load(open(os.path.join(REPO, "tests", "golden", "big.json")))["config1_2^16_u32"]


def _sha(np, x) -> str:
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()


def _median_s(fn, reps: int) -> float:
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


def config1_cpu(ls):
    """BASELINE config 1 on the CPU reference path (part of cpu_baseline): n=2^16 uniform
    uint32 keys (main.cpp's largest size) sorted by std::sort (the oracle, one core) and
    by order_with_trust (rocThrust's host sort, lab.cu:404-406; CPU, F7), each checked
    against the committed fixture (tests/golden/big.json)."""
    import numpy as np
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as O  # test infrastructure: the CPU baseline leg only
    c = _config1_fixture()
    n = 1 << c["log2n"]
    a = O.gen(n, c["seed"], c["dist"])
    ok = _sha(np, a) == c["sha256_input"] and _sha(np, O.sort_u32(a)) == c["sha256_sorted_u32"]
    t_std = O.time_sort_u32(a, threads=1, reps=200) / 200
    b = a.view(np.int32).copy()

    def trust():
        np.copyto(b, a.view(np.int32))
        ls.order_with_trust(b)
    t_trust = _median_s(trust, 50)
    ok = ok and _sha(np, b) == c["sha256_sorted_i32"]
    return {"workload": "n=2^16 uniform uint32 (BASELINE config 1)", "cores": 1,
            "verified": "fixture" if ok else "FIXTURE MISMATCH",
            "std_sort": {"ms": round(t_std * 1e3, 4), "Mkeys_s": round(n / t_std / 1e6, 2)},
            "order_with_trust": {"ms": round(t_trust * 1e3, 4), "Mkeys_s": round(n / t_trust / 1e6, 2)},
            "published_reference": {"std_sort_ms": 2.383, "thrust_host_ms": 0.384,
                                    "source": "Informe p.5 (BASELINE.md), other host, for context"}}


def config1_gpu(ls, torch, dev, stream):
    """BASELINE config 1's array through the GPU: order_array (the drop-in, host pointer
    in/out: H2D + sort + D2H, the call main.cpp:28 times) and the device-resident sort;
    both checked against the committed fixture's SHA-256 (no CPU sort)."""
    import numpy as np
    c = _config1_fixture()
    n = 1 << c["log2n"]
    src = torch.empty(n, dtype=torch.int32, device=dev)
    ls.fill(src, n, c["seed"], c["dist"], stream=stream)
    torch.cuda.synchronize()
    a = src.cpu().numpy()
    ok = _sha(np, a) == c["sha256_input"]
    h = a.copy()

    def oa():
        np.copyto(h, a)
        ls.order_array(h)
    oa()
    t_oa = _median_s(oa, 50)
    ok = ok and _sha(np, h) == c["sha256_sorted_i32"]
    out = torch.empty_like(src)
    ws = torch.empty(max(ls.workspace_bytes(n, "auto"), 256), dtype=torch.uint8, device=dev)
    for _ in range(5):
        ls.sort_device(src, out, n, key="u32", algo="auto", workspace=ws, stream=stream)
    torch.cuda.synchronize()
    reps = 200
    t0 = time.perf_counter()
    for _ in range(reps):
        ls.sort_device(src, out, n, key="u32", algo="auto", workspace=ws, stream=stream)
    torch.cuda.synchronize()
    t_dev = (time.perf_counter() - t0) / reps
    ok = ok and _sha(np, out.cpu().numpy().view(np.uint32)) == c["sha256_sorted_u32"]
    return {"workload": "n=2^16 uniform uint32 (BASELINE config 1) through the GPU",
            "verified": "fixture" if ok else "FIXTURE MISMATCH",
            "order_array_host_pointer": {"ms": round(t_oa * 1e3, 4), "Mkeys_s": round(n / t_oa / 1e6, 2)},
            "sort_device": {"ms": round(t_dev * 1e3, 4), "Mkeys_s": round(n / t_dev / 1e6, 2)},
            "published_reference_order_array_ms": 1.066}


def host_fingerprint(np, a):
    """count, sum and sum of squares (mod 2^64) of the keys as uint32, in 64 Mi-key chunks"""
    u = a.view(np.uint32)
    s1 = s2 = 0
    for i in range(0, u.size, 1 << 26):
        c = u[i:i + (1 << 26)].astype(np.uint64)
        s1 = (s1 + int(c.sum(dtype=np.uint64))) & (2**64 - 1)
        s2 = (s2 + int((c * c).sum(dtype=np.uint64))) & (2**64 - 1)
    return u.size, s1, s2


def host_sorted(np, a) -> bool:
    v = a  # int32: order_array's signed order
    for i in range(0, v.size - 1, 1 << 26):
        c = v[i:i + (1 << 26) + 1]
        if not bool((c[1:] >= c[:-1]).all()):
            return False
    return True


def host_leg_main(args) -> None:
    """Child process of the host_path leg: one pageable int32 host array sorted in place
    through labsort_sort_host (1 GPU) and labsort_sort_host_multi (devices 0..N-1)."""
    import numpy as np
    import torch
    sys.path.insert(0, REPO)
    ls = importlib.import_module(PKG_NAME)
    n = 1 << args.host_log2n
    t = torch.empty(n, dtype=torch.int32, device="cuda:0")
    ls.fill(t, n, SEED + 5, "u31")  # the reference's keys: non-negative int (main.cpp rand())
    torch.cuda.synchronize()
    src = t.cpu().numpy()
    del t
    torch.cuda.empty_cache()
    fp = host_fingerprint(np, src)
    work = np.empty_like(src)
    out = {"n": n, "key": "i32 (order_array)", "input": "pageable host array, u31 keys (main.cpp's rand())",
           "note": "PCIe-inclusive: H2D + sort + D2H of a host int*, in place (never `value`)"}

    def timed(fn, reps):
        ts = []
        for _ in range(reps):
            np.copyto(work, src)
            t0 = time.perf_counter()
            fn(work)
            ts.append(time.perf_counter() - t0)
        ok = host_sorted(np, work) and host_fingerprint(np, work) == fp
        return sorted(ts)[len(ts) // 2], ok

    if args.host_leg == "peer":
        el, ok = timed(lambda a: ls.sort_host(a, algo="auto"), 3)
        out["single_gpu"] = {"ms": round(el * 1e3, 3), "Mkeys_s": round(n / el / 1e6, 2), "verified": ok,
                             "call": "labsort_sort_host (order_array; pipelined chunks from 2^27 keys)"}
        # BASELINE config 5's own partition on this GPU: 8 ranks sharing it (peer copies
        # stand in for xGMI): chunked H2D per rank, splitters, exchange, merge, ranged D2H
        el, ok = timed(lambda a: ls.sort_host_ranks(a, [0] * 8, transport="peer"), 3)
        ph, sent = ls.multi_timing()
        counts = ls.multi_range_counts(8)
        out["config5_8ranks_one_gpu"] = {
            "ms": round(el * 1e3, 3), "Mkeys_s": round(n / el / 1e6, 2), "verified": ok,
            "call": "labsort_sort_host_ranks(devices [0]*8, peer): the 8-rank schedule on one GPU",
            "phases_ms": {k: round(v, 3) for k, v in ph.items()}, "max_sent_bytes": sent,
            "max_range_over_share": round(max(counts) / (n / 8), 4)}
    if args.gpus > 1 and torch.cuda.device_count() < args.gpus:
        out[f"error_{args.host_leg}"] = f"{torch.cuda.device_count()} devices visible, {args.gpus} needed"
    elif args.gpus > 1:
        devs = list(range(args.gpus))
        if args.host_leg == "rccl":
            ls.set_comm_timeout(30.0)  # (a transport problem ends this leg in 30 s, well inside its 100 s limit)
        try:
            el, ok = timed(lambda a: ls.sort_host_ranks(a, devs, transport=args.host_leg), 3)
        except ls.LabsortError as e:
            out[f"error_{args.host_leg}"] = str(e)
            print(json.dumps(out), flush=True)
            return
        ph, sent = ls.multi_timing()
        out[f"multi_gpu_{args.host_leg}"] = {
            "n_gpus": args.gpus, "ms": round(el * 1e3, 3), "Mkeys_s": round(n / el / 1e6, 2), "verified": ok,
            "call": "labsort_sort_host_ranks(devices 0..N-1, " + (
                "RCCL send/recv: what LABSORT_GPUS=N order_array uses)" if args.host_leg == "rccl"
                else "hipMemcpyPeerAsync exchange)"),
            "phases_ms": {k: round(v, 3) for k, v in ph.items()}, "max_sent_bytes": sent}
    print(json.dumps(out), flush=True)


def host_leg(args, timeout_s: int = 100):
    """Run the host_path leg in child processes: each opens the GPUs it uses itself, and a
    hang or fault there ends only that child (reported as an error).  First the single-GPU
    sort and the multi-GPU schedule with peer copies, then (N > 1) the same schedule over
    RCCL, so an RCCL problem cannot cost the other numbers."""
    import subprocess
    drop = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
            "ROLE_RANK", "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")
    env = {k: v for k, v in os.environ.items() if k not in drop}
    out = {}
    for xfer in ("peer", "rccl") if args.gpus > 1 else ("peer",):
        cmd = [sys.executable, os.path.abspath(__file__), "--host-leg", xfer, "--gpus", str(args.gpus),
               "--host-log2n", str(args.host_log2n)]
        try:
            r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout_s)
        except subprocess.TimeoutExpired:
            out[f"error_{xfer}"] = f"timed out after {timeout_s} s"
            continue
        got = None
        for ln in reversed(r.stdout.splitlines()):
            if ln.startswith("{"):
                got = json.loads(ln)
                break
        if got is None:
            out[f"error_{xfer}"] = f"exit {r.returncode}: {r.stderr.strip()[-400:]}"
        else:
            out.update(got)
    return out


def dist_leg(torch, ls, dmod, args, dev, cdev, stream, rank, world, sizes, seed, dcomm=None, comm=None):
    """One N > 1 measurement: rank r sorts its shard of sizes[r] keys (keys first ..
    first + sizes[r] of the generator: the shards are the global array's pieces) as one
    step of the distributed merge sort, W untimed + K timed steps between barriers, the
    max over ranks of the elapsed time; then the global result is verified (every range
    sorted, ranges in rank order, the same digit histograms and sum as the input)."""
    import torch.distributed as dist
    key = "u32"
    m, first = sizes[rank], sum(sizes[:rank])
    src = torch.empty(max(m, 1), dtype=torch.int32, device=dev)
    if m:
        ls.fill(src, m, SEED + 5, args.dist, first=first, stream=stream)
    torch.cuda.synchronize()
    if args.exchange == "splitters":
        def step():  # the product: labsort_dist_sort (csrc/dist_plan.h's schedule)
            ptr, cnt, _ = dcomm.sort(src, m, key=key, stream=stream)
            return ptr, cnt
    else:
        ops = dmod.HipOps(ls, key=key, local_algo="radix", stream=stream)

        def step():
            with torch.cuda.stream(stream):
                return dmod.dist_sort(src[:m], ops, copy_input=True, comm=comm)
    for _ in range(args.warmup):
        res = step()
    torch.cuda.synchronize()
    if args.exchange != "splitters":
        comm.sent_bytes, comm.p2p_rounds, comm.exchange_s = 0, 0, 0.0
        comm.timed = True
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    dist.barrier()
    elapsed = time.perf_counter() - t0
    tt = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed = float(tt.item())
    if args.exchange == "splitters":  # the last step's range, viewed in the comm's buffer
        res = ls.DistComm.view(*res, owner=dcomm)
        dphase, dsent = dcomm.timing()
        dcoll = dcomm.collectives()
    # global check: every range sorted, boundaries ordered, multiset preserved
    nres = res.numel()
    cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    ls.count_descents(res, nres, cnt, key=key)
    edges = ((torch.stack([res[0], res[-1]]).to(torch.int64) & 0xFFFFFFFF)).to(cdev) if nres else \
        torch.tensor([2**33, -1], dtype=torch.int64, device=cdev)  # empty range: neutral for the order check
    allg = [torch.empty_like(edges) for _ in range(world)]
    dist.all_gather(allg, edges)
    h_in = torch.zeros(1024, dtype=torch.int32, device=dev)
    h_out = torch.zeros(1024, dtype=torch.int32, device=dev)
    ls.histogram(src, m, h_in, key=key)
    ls.histogram(res, nres, h_out, key=key)
    s_in = (src[:m].to(torch.int64) & 0xFFFFFFFF).sum()
    s_out = (res.to(torch.int64) & 0xFFFFFFFF).sum()
    red = torch.stack([s_in, s_out]).to(cdev)
    h_in, h_out = h_in.to(cdev), h_out.to(cdev)
    dist.all_reduce(h_in)
    dist.all_reduce(h_out)
    dist.all_reduce(red)
    ok = int(cnt.item()) == 0 and torch.equal(h_in, h_out) and int(red[0]) == int(red[1])
    lastmax = -1
    for e in allg:  # ranges in rank order: each range's first key >= every earlier key
        if int(e[0]) > 2**32:
            continue
        ok = ok and int(e[0]) >= lastmax
        lastmax = int(e[1])
    okt = torch.tensor([1 if ok else 0], dtype=torch.int32, device=cdev)
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    ok = bool(okt.item())
    # exchange statistics: max over ranks (last step); the plan's work and wait
    ph_names = ("local_sort", "plan", "plan_work", "plan_wait", "exchange", "merge")
    if args.exchange == "splitters":
        vals = [float(dsent), dphase["exchange"] * 1e6, 1.0] + [dphase[k] * 1e6 for k in ph_names]
    else:
        vals = [comm.sent_bytes / args.steps, comm.exchange_s * 1e9 / args.steps, comm.p2p_rounds / args.steps] + \
            [0.0] * len(ph_names)
    st = torch.tensor(vals, dtype=torch.float64, device=cdev)
    dist.all_reduce(st, op=dist.ReduceOp.MAX)
    sent, exs, rounds = float(st[0]), float(st[1]) / 1e9, float(st[2])
    links = world - 1 if args.exchange == "splitters" else 1
    xgmi = {"bytes_sent_per_rank_per_step": int(sent), "p2p_rounds_per_step": rounds,
            "exchange_ms_per_step": round(exs * 1e3, 4), "links_per_round": links,
            "per_link_GBps": round(sent / links / exs / 1e9, 2) if exs > 0 else None,
            "note": ("max over ranks, last step; exchange = device time of the grouped ncclSend/ncclRecv "
                     "(labsort_dist_timing); plan_wait = time inside the plan's collectives (waiting for "
                     "the slowest rank), plan_work = the rest" if args.exchange == "splitters" else
                     "max over ranks; exchange time is host wall time around the point-to-point calls")}
    if args.exchange == "splitters":
        xgmi["phases_ms_last_step"] = {k: round(float(st[3 + i]) / 1e6, 4) for i, k in enumerate(ph_names)}
        # every rank's arrival at / return from each collective (ms since its call started)
        mine = torch.tensor([v for k in ls.COLLECTIVES for v in dcoll[k]], dtype=torch.float64, device=cdev)
        allc = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allc, mine)
        xgmi["collectives_ms_last_step"] = {
            k: [[round(float(allc[r][2 * i]), 3), round(float(allc[r][2 * i + 1]), 3)] for r in range(world)]
            for i, k in enumerate(ls.COLLECTIVES) if any(float(allc[r][2 * i]) >= 0 for r in range(world))}
    del src, res
    return {"elapsed": elapsed, "ok": ok, "xgmi": xgmi, "keys": sum(sizes)}


def dist_main(args, torch, ls, world, rank, dev):
    """N > 1 (one process per GPU under torch.distributed.run): BASELINE config 5 -- a
    2^total-log2n-key array (default 2^30) partitioned over the N ranks (2^30 / N keys
    each: strong scaling) and sorted by the product's distributed merge sort; then, as a
    secondary field, the same schedule with 2^log2n keys per rank (weak scaling)."""
    import torch.distributed as dist
    cdev = dev if args.backend == "nccl" else torch.device("cpu")  # where collectives' tensors live
    if args.backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    dmod = importlib.import_module(PKG_NAME + ".dist")
    stream = torch.cuda.Stream(device=dev)
    dcomm = dmod.make_comm(ls, backend=args.backend) if args.exchange == "splitters" else None
    comm = None
    if args.exchange != "splitters":
        comm = dmod.P2PComm() if args.backend == "nccl" else dmod.HostStagedComm()
    total = 1 << args.total_log2n
    strong = dist_leg(torch, ls, dmod, args, dev, cdev, stream, rank, world,
                      [total * (r + 1) // world - total * r // world for r in range(world)], SEED + 5, dcomm, comm)
    weak = None
    if not args.no_weak:
        weak = dist_leg(torch, ls, dmod, args, dev, cdev, stream, rank, world, [1 << args.log2n] * world,
                        SEED + 5, dcomm, comm)
    if not (strong["ok"] and (weak is None or weak["ok"])):
        print(f"bench.py: rank {rank}: OUTPUT CHECK FAILED (sort result is not a sorted permutation)", file=sys.stderr)
        sys.exit(3)
    dist.barrier()
    if dcomm is not None:
        try:  # (a teardown error is reported, not allowed to lose the measured line)
            dcomm.close()
        except Exception as e:  # noqa: BLE001
            print(f"bench.py: rank {rank}: communicator teardown: {e}", file=sys.stderr)
    dist.destroy_process_group()
    # the host-pointer leg runs once every rank is done with its GPU
    hostp = host_leg(args) if rank == 0 and not args.no_host_path and args.backend == "nccl" else None
    if rank != 0:
        return
    how = ("splitter exchange (labsort_dist_sort: pairwise ncclSend/ncclRecv to all peers at once, merge of "
           "the received runs)" if args.exchange == "splitters" else "bitonic pairwise merge-split network")
    line = {
        "metric": "Mkeys/s sorting uint32, n=2^28, 1 GPU (+ merge-sort at 2/4/8)",
        "value": round(strong["keys"] * args.steps / strong["elapsed"] / 1e6, 2), "unit": "Mkeys/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(strong["elapsed"] / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (counter-based splitmix64 generator on device)",
        "config": {"workload": f"BASELINE config 5: n=2^{args.total_log2n} uint32 merge sort partitioned across "
                               f"{world} GPUs (2^{args.total_log2n}/{world} keys per rank): local radix sort + {how} "
                               f"over {'RCCL/xGMI' if args.backend == 'nccl' else 'gloo host collectives (rehearsal)'}",
                   "n_total": strong["keys"], "n_per_gpu": strong["keys"] // world, "algo": "merge",
                   "local_algo": "radix", "key": "u32", "dist": args.dist,
                   "parallelism": f"{world} ranks, {'RCCL' if args.backend == 'nccl' else 'gloo'} {args.exchange} exchange"},
        "verified": "sorted permutation (descents, digit histograms, sums), ranges in rank order",
        "xgmi": strong["xgmi"], "roofline": None, "cpu_baseline": None,
    }
    if weak:
        line["weak"] = {"workload": f"the same schedule with 2^{args.log2n} keys per GPU (weak scaling)",
                        "value": round(weak["keys"] * args.steps / weak["elapsed"] / 1e6, 2), "unit": "Mkeys/s",
                        "ms_per_step": round(weak["elapsed"] / args.steps * 1e3, 4), "scaling": "weak",
                        "xgmi": weak["xgmi"]}
    if hostp:
        line["host_path"] = hostp
    print(json.dumps(line), flush=True)


def launch_ranks(args, torch) -> int:
    """`python bench.py --gpus N` (N > 1) without torch.distributed.run around it: start the
    N ranks here, as ONE child process tree (torch.distributed.run, 127.0.0.1 rendezvous)
    before this process touches the GPU (torch.cuda.device_count() does not initialise it),
    relay their output, and return non-zero unless rank 0 printed its config-5 line.  A
    deadline (--launch-timeout) ends the whole tree (SIGTERM, then SIGKILL); torch.distributed.run
    itself ends every rank when one fails.  With --backend nccl every rank needs its own GPU:
    fewer visible devices than N is refused at once."""
    import signal
    import socket
    import subprocess
    import threading
    ndev = torch.cuda.device_count()
    if args.backend == "nccl" and ndev < args.gpus:
        print(f"bench.py: --gpus {args.gpus} with --backend nccl needs {args.gpus} GPUs, {ndev} visible "
              "(one rank per GPU); --backend gloo rehearses several ranks on one GPU", file=sys.stderr)
        return 2
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    drop = ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
            "ROLE_RANK", "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["PYTHONUNBUFFERED"] = "1"
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    def on_parent_death():  # (in the child: if this launcher is killed, torch.distributed.run gets SIGTERM
        # and ends its ranks, instead of leaving them on the GPUs)
        try:
            import ctypes
            ctypes.CDLL("libc.so.6", use_errno=True).prctl(1, signal.SIGTERM)  # PR_SET_PDEATHSIG
        except OSError:
            pass
    p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, start_new_session=True,
                         preexec_fn=on_parent_death)
    expired = threading.Event()

    def deadline():
        expired.set()
        for sig, wait in ((signal.SIGTERM, 10), (signal.SIGKILL, 0)):
            try:
                os.killpg(p.pid, sig)
            except ProcessLookupError:
                return
            try:
                p.wait(timeout=wait) if wait else None
                return
            except subprocess.TimeoutExpired:
                continue
    timer = threading.Timer(args.launch_timeout, deadline)
    timer.daemon = True
    timer.start()
    line = None
    try:
        for ln in p.stdout:
            sys.stdout.write(ln)
            sys.stdout.flush()
            if ln.startswith("{"):
                try:
                    line = json.loads(ln)
                except json.JSONDecodeError:
                    pass
        rc = p.wait()
    finally:
        timer.cancel()
        if p.poll() is None:
            deadline()
    if expired.is_set():
        print(f"bench.py: the {args.gpus} ranks did not finish within {args.launch_timeout:.0f} s; ended them",
              file=sys.stderr)
        return 124
    if rc != 0:
        print(f"bench.py: the ranks' launcher exited {rc}", file=sys.stderr)
        return rc if rc > 0 else 1
    if not line or line.get("n_gpus") != args.gpus:
        print("bench.py: rank 0 printed no result line", file=sys.stderr)
        return 1
    return 0


def main():
    args = parse()
    if args.host_leg:
        return host_leg_main(args)
    import torch

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args, torch))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    local = local % max(torch.cuda.device_count(), 1)  # ranks share a device only in the gloo test mode
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if REPO not in sys.path:
        sys.path.insert(0, REPO)
    ls = importlib.import_module(PKG_NAME)
    if world > 1:
        return dist_main(args, torch, ls, world, rank, dev)

    n = 1 << args.log2n
    key = "u32"
    stream = torch.cuda.Stream(device=dev)
    ws = None

    if args.algo == "pairs":
        src = torch.empty(n, dtype=torch.int32, device=dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        vsrc = torch.arange(n, dtype=torch.int32, device=dev)
        vout = torch.empty(n, dtype=torch.int32, device=dev)
        ws = torch.empty(max(ls.pairs_workspace_bytes(n, args.pair_algo), 256), dtype=torch.uint8, device=dev)
        ls.fill(src, n, SEED + 3, args.dist, stream=stream)

        def step():
            ls.sort_pairs_device(src, vsrc, out, vout, n, key=key, algo=args.pair_algo, workspace=ws, stream=stream)
            return out
    else:
        src = torch.empty(n, dtype=torch.int32, device=dev)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        ws = torch.empty(max(ls.workspace_bytes(n, args.algo), 256), dtype=torch.uint8, device=dev)
        ls.fill(src, n, SEED + 3, args.dist, stream=stream)

        def step():
            ls.sort_device(src, out, n, key=key, algo=args.algo, workspace=ws, stream=stream)
            return out

    def status():
        """the kernels' own error report for the last sort (raises LabsortError)"""
        if args.algo == "pairs":
            ls.pairs_workspace_status(ws, n, args.pair_algo, stream=stream)
        else:
            ls.workspace_status(ws, n, args.algo, stream=stream)

    torch.cuda.synchronize()
    for _ in range(args.warmup):
        res = step()
    torch.cuda.synchronize()
    status()

    dom = "onesweep" if args.algo in ("radix", "radix1") or (args.algo == "pairs" and args.pair_algo == "radix") \
        else "merge"
    if args.algo == "radix" and ls.radix_impl(n) == "gather":
        dom = "gsweep"  # the gathered passes (2^16 <= n < 2^25)
    ls.timing_enable(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res = step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    k_ms, k_cnt = ls.timing_read(dom)
    ls.timing_enable(False)
    elapsed = t1 - t0
    status()

    ok, desc = verify(torch, ls, src, res, n, key)
    if ok and args.algo == "pairs":
        # each payload is its key's input index: the gather reproduces the output keys,
        # and equal keys keep ascending indices (stable)
        idx = vout.to(torch.int64)
        ok = bool((idx >= 0).all()) and bool((idx < n).all()) and torch.equal(src[idx], res)
        if ok and n > 1:
            ok = bool(((vout[1:] > vout[:-1]) | (res[1:] != res[:-1])).all())
        del idx
    if not ok:
        print(f"bench.py: rank {rank}: OUTPUT CHECK FAILED (sort result is not a sorted permutation)",
              file=sys.stderr)
        sys.exit(3)

    # config 4 beside the headline: the merge sort of the same device input (N = 1,
    # radix headline only); its own verification, status check and kernel timings
    merge_leg = None
    if args.algo == "radix" and not args.no_merge:
        mws = torch.empty(max(ls.workspace_bytes(n, "merge"), 256), dtype=torch.uint8, device=dev)
        mout = torch.empty_like(src)

        def mstep():
            ls.sort_device(src, mout, n, key=key, algo="merge", workspace=mws, stream=stream)

        for _ in range(args.warmup):
            mstep()
        torch.cuda.synchronize()
        ls.timing_enable(True)
        m0 = time.perf_counter()
        for _ in range(args.steps):
            mstep()
        torch.cuda.synchronize()
        m1 = time.perf_counter()
        mp_ms, mp_cnt = ls.timing_read("merge")
        m4_ms, m4_cnt = ls.timing_read("merge4")
        ts_ms, ts_cnt = ls.timing_read("tile_sort")
        ls.timing_enable(False)
        ls.workspace_status(mws, n, "merge", stream=stream)
        mok, _ = verify(torch, ls, src, mout, n, key)
        if not mok:
            print("bench.py: MERGE OUTPUT CHECK FAILED", file=sys.stderr)
            sys.exit(3)
        mavg = mp_ms / mp_cnt if mp_cnt else None
        m4avg = m4_ms / m4_cnt if m4_cnt else None
        tavg = ts_ms / ts_cnt if ts_cnt else None
        mtraffic, msrc = pmc_traffic("merge", n)
        m4traffic, m4src = pmc_traffic("merge4", n)
        ttraffic, _ = pmc_traffic("tile_sort", n)

        def pass_roofline(kernel, avg, traffic, src):
            return {"bound": "hbm", "kernel": kernel, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "avg_launch_ms": round(avg, 5) if avg else None,
                    "achieved": round(8.0 * n / (avg * 1e-3) / 1e9, 1) if avg else None,
                    "frac": round(8.0 * n / (avg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if avg else None,
                    "algorithmic_bytes_per_launch": 8.0 * n, "traffic": traffic, "traffic_source": src}
        # dominant merge kernel: the four-way pass (two merge levels per read and write of the
        # keys; its launch = k_m4_rank + k_m4_merge), the pairwise pass when no four-way ran
        four = bool(m4_cnt)
        merge_leg = {
            "workload": f"LDS tile sort + merge passes (four-way, one pairwise for an odd level count) of the same "
                        f"2^{args.log2n} device-resident keys (BASELINE config 4)",
            "value": round(n * args.steps / (m1 - m0) / 1e6, 2), "unit": "Mkeys/s",
            "ms_per_step": round((m1 - m0) / args.steps * 1e3, 4),
            "passes_per_sort": (mp_cnt + m4_cnt) // max(args.steps, 1),
            "four_way_passes_per_sort": m4_cnt // max(args.steps, 1),
            "verified": "sorted permutation (descents, digit histograms, sums)",
            "roofline": (pass_roofline("k_m4_rank + k_m4_merge", m4avg, m4traffic, m4src) if four
                         else pass_roofline("k_merge_pass_p", mavg, mtraffic, msrc)),
            "pairwise_pass": pass_roofline("k_merge_pass_p", mavg, mtraffic, msrc) if four and mavg else None,
            "tile_sort": {"kernel": "k_tile_sort", "avg_launch_ms": round(tavg, 5) if tavg else None,
                          "achieved": round(8.0 * n / (tavg * 1e-3) / 1e9, 1) if tavg else None,
                          "frac": round(8.0 * n / (tavg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if tavg else None,
                          "traffic": ttraffic},
        }
        del mws, mout

    # BASELINE config 2 beside the headline: 2^20 keys, radix (the gathered passes at this
    # size), device-resident, verified; launch-bound, so reported as time per sort
    config2 = None
    if args.algo == "radix" and not args.no_merge and n > (1 << 20):
        n2 = 1 << 20
        s2 = torch.empty(n2, dtype=torch.int32, device=dev)
        o2 = torch.empty_like(s2)
        w2 = torch.empty(max(ls.workspace_bytes(n2, "radix"), 256), dtype=torch.uint8, device=dev)
        ls.fill(s2, n2, SEED + 2, args.dist, stream=stream)
        for _ in range(3):
            ls.sort_device(s2, o2, n2, key=key, algo="radix", workspace=w2, stream=stream)
        torch.cuda.synchronize()
        reps = 50
        c0 = time.perf_counter()
        for _ in range(reps):
            ls.sort_device(s2, o2, n2, key=key, algo="radix", workspace=w2, stream=stream)
        torch.cuda.synchronize()
        c1 = time.perf_counter()
        ls.workspace_status(w2, n2, "radix", stream=stream)
        ok2, _ = verify(torch, ls, s2, o2, n2, key)
        if not ok2:
            print("bench.py: CONFIG 2 OUTPUT CHECK FAILED", file=sys.stderr)
            sys.exit(3)
        config2 = {"workload": "n=2^20 uint32 radix sort, device-resident (BASELINE config 2)",
                   "impl": ls.radix_impl(n2), "ms_per_sort": round((c1 - c0) / reps * 1e3, 4),
                   "value": round(n2 * reps / (c1 - c0) / 1e6, 2), "unit": "Mkeys/s",
                   "verified": "sorted permutation (descents, digit histograms, sums)"}
        del s2, o2, w2

    # SURVEY 8f row 4 beside the headline: the stable key/value radix sort of the same keys
    # with 4-byte payloads (each its input index), verified as the pairs run is
    pairs_leg = None
    if args.algo == "radix" and not args.no_merge:
        vin = torch.arange(n, dtype=torch.int32, device=dev)
        pko = torch.empty_like(src)
        pvo = torch.empty_like(src)

        def prun(palgo, cls):
            """time args.steps key/value sorts with `palgo`; verify; (ms per step, cls launch mean)"""
            pws = torch.empty(max(ls.pairs_workspace_bytes(n, palgo), 256), dtype=torch.uint8, device=dev)

            def pstep():
                ls.sort_pairs_device(src, vin, pko, pvo, n, key=key, algo=palgo, workspace=pws, stream=stream)

            for _ in range(args.warmup):
                pstep()
            torch.cuda.synchronize()
            ls.timing_enable(True)
            p0 = time.perf_counter()
            for _ in range(args.steps):
                pstep()
            torch.cuda.synchronize()
            p1 = time.perf_counter()
            c_ms, c_cnt = ls.timing_read(cls)
            ls.timing_enable(False)
            ls.pairs_workspace_status(pws, n, palgo, stream=stream)
            del pws
            pok, _ = verify(torch, ls, src, pko, n, key)
            if pok:
                idx = pvo.to(torch.int64)
                pok = bool((idx >= 0).all()) and bool((idx < n).all()) and torch.equal(src[idx], pko)
                if pok and n > 1:
                    pok = bool(((pvo[1:] > pvo[:-1]) | (pko[1:] != pko[:-1])).all())
                del idx
            if not pok:
                print(f"bench.py: KEY/VALUE OUTPUT CHECK FAILED ({palgo})", file=sys.stderr)
                sys.exit(3)
            return (p1 - p0) / args.steps * 1e3, (c_ms / c_cnt if c_cnt else None)

        pms, pavg = prun("radix", "onesweep")
        mms, mavg = prun("merge", "merge4")
        pairs_leg = {"workload": f"stable key/value LSD radix (4-byte payloads) of the same 2^{args.log2n} keys",
                     "value": round(n / (pms * 1e-3) / 1e6, 2), "unit": "Mpairs/s",
                     "ms_per_step": round(pms, 4),
                     "verified": "sorted, payload = input index of its key, equal keys in input order",
                     "roofline": {"bound": "hbm", "kernel": "k_onesweep_p<true> (key/value)", "peak": HBM_PEAK_GBS,
                                  "unit": "GB/s", "avg_launch_ms": round(pavg, 5) if pavg else None,
                                  "achieved": round(16.0 * n / (pavg * 1e-3) / 1e9, 1) if pavg else None,
                                  "frac": round(16.0 * n / (pavg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if pavg else None,
                                  "algorithmic_bytes_per_launch": 16.0 * n},
                     "merge": {"workload": "stable key/value merge sort (tile sort + four-way passes carrying the payloads)",
                               "value": round(n / (mms * 1e-3) / 1e6, 2), "unit": "Mpairs/s", "ms_per_step": round(mms, 4),
                               "four_way_pass_ms": round(mavg, 5) if mavg else None,
                               "verified": "sorted, payload = input index of its key, equal keys in input order"}}
        del vin, pko, pvo

    config1 = None
    if args.algo == "radix" and not args.no_merge:
        config1 = config1_gpu(ls, torch, dev, stream)
        if config1["verified"] != "fixture":
            print("bench.py: CONFIG 1 OUTPUT CHECK FAILED", file=sys.stderr)
            sys.exit(3)

    value = n * args.steps / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3
    # the host-pointer leg (PCIe-inclusive, child processes)
    hostp = host_leg(args) if not args.no_host_path else None

    # the copy ceiling: the library's streaming copy (labsort_copy: 16-B nontemporal loads
    # and stores in 16384-word tiles, one workgroup per CU) of the same n keys, each of 5
    # launches timed by HIP events on the stream it runs on; the median launch
    cp = torch.empty_like(src)
    for _ in range(2):
        ls.copy(src, cp, n, stream=stream)
    times = []
    for _ in range(5):
        ls.timing_enable(True)
        ls.copy(src, cp, n, stream=stream)
        torch.cuda.synchronize()
        times.append(ls.timing_read("copy")[0])
        ls.timing_enable(False)
    copy_ms = sorted(times)[len(times) // 2]
    copy_gbs = 8.0 * n / (copy_ms * 1e-3) / 1e9
    copy_ok = torch.equal(cp, src)
    del cp

    avg_ms = k_ms / k_cnt if k_cnt else None
    per_launch_bytes = 16.0 * n if args.algo == "pairs" else 8.0 * n  # key (+ payload) read + written
    achieved = per_launch_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms else None
    traffic, tsrc = pmc_traffic(dom, n)
    roofline = {"bound": "hbm", "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                "traffic": traffic, "kernel": ("k_onesweep_p" if dom == "onesweep" and args.algo == "radix" else
                                               "k_gsweep" if dom == "gsweep" else
                                               "k_onesweep_p<true>" if args.algo == "pairs" and dom == "onesweep"
                                               else f"k_{dom}"), "launches": k_cnt,
                "avg_launch_ms": round(avg_ms, 5) if avg_ms else None,
                "algorithmic_bytes_per_launch": per_launch_bytes, "traffic_source": tsrc}
    roofline["copy_ceiling"] = {
        "value": round(copy_gbs, 1), "unit": "GB/s", "frac": round(achieved / copy_gbs, 4) if achieved else None,
        "ms": round(copy_ms, 5), "verified": bool(copy_ok),
        "probe": "labsort_copy of the same n keys (16-B nontemporal loads and stores, 16384-word tiles, one "
                 "1024-thread workgroup per CU), median of 5 event-timed launches, after the timed region"}
    cpu = None
    if not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds, n, ls)
        cpu["config1"] = config1_cpu(ls)
    wl = {"radix": "LSD radix sort (8-bit digits, onesweep)", "merge": "LDS tile sort + merge-path passes",
          "radix1": "LSD radix with 1-bit split passes (letra.pdf)",
          "pairs": "stable key/value sort (uint32 key + uint32 index payload): " + (
              "8-bit LSD onesweep passes" if args.pair_algo == "radix" else "LDS tile sort + merge-path passes")
          }[args.algo]
    line = {
        "metric": "Mkeys/s sorting uint32, n=2^28, 1 GPU (+ merge-sort at 2/4/8)",
        "value": round(value, 2), "unit": "Mkeys/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (counter-based splitmix64 generator on device)",
        "config": {"workload": f"{wl}, n=2^{args.log2n} uint32 {args.dist}, device-resident (BASELINE config 3)",
                   "n_per_gpu": n, "algo": args.algo, "key": key, "dist": args.dist, "parallelism": "single GPU"},
        "verified": "sorted permutation (descents, digit histograms, sums)" + (
            "; payloads gather the output keys, stable" if args.algo == "pairs" else ""),
        "roofline": roofline, "cpu_baseline": cpu,
    }
    for leg in (merge_leg and merge_leg["roofline"], merge_leg and merge_leg["tile_sort"],
                merge_leg and merge_leg.get("pairwise_pass"), pairs_leg and pairs_leg["roofline"]):  # each leg's dominant kernel against the same copy
        if leg and leg.get("achieved"):
            leg["copy_frac"] = round(leg["achieved"] / copy_gbs, 4)
    if merge_leg:
        line["merge"] = merge_leg
    if config1:
        line["config1"] = config1
    if config2:
        line["config2"] = config2
    if pairs_leg:
        line["pairs"] = pairs_leg
    if hostp:
        line["host_path"] = hostp
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
