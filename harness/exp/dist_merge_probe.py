"""Diagnostic: the multi-GPU exchange's merge step on one GPU.  p sorted runs of
2^28/p keys back to back (what a rank holds after the splitter exchange), merged by
(a) the Python tree of labsort_merge calls (HipOps(kway=False)), (b) labsort_merge_runs
(HipOps default): log2 p levels of merge-path passes over explicit pairs of runs, and
(c) labsort_merge_runs with LABSORT_MERGE_RUNS=kway (one K-way pass, kmerge.hip).
Median ms of 10 after warm-up; the three outputs must be equal."""
import importlib, json, os, sys, time
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
import torch
PKG = "radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd"
ls = importlib.import_module(PKG)
D = importlib.import_module(PKG + ".dist")
n = 1 << int(os.environ.get("LOG2N", "28"))
for p in (2, 4, 8):
    m = n // p
    buf = torch.empty(n, dtype=torch.int32, device="cuda")
    ls.fill(buf, n, 77, "u32")
    ws = torch.empty(ls.workspace_bytes(m, "radix"), dtype=torch.uint8, device="cuda")
    for q in range(p):
        ls.sort_device(buf[q * m:(q + 1) * m], buf[q * m:(q + 1) * m], m, workspace=ws)
    offs = [q * m for q in range(p + 1)]
    row = {"p": p, "n": n}
    outs = []
    for mode in ("tree", "passes", "kway"):
        kway = mode != "tree"
        if mode == "kway":
            os.environ["LABSORT_MERGE_RUNS"] = "kway"
        else:
            os.environ.pop("LABSORT_MERGE_RUNS", None)
        ops = D.HipOps(ls, kway=kway)
        for _ in range(2):
            ops.merge_runs(buf, offs)
        torch.cuda.synchronize()
        ts = []
        for _ in range(10):
            t0 = time.perf_counter()
            out = ops.merge_runs(buf, offs)
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        ts.sort()
        row[mode + "_ms"] = round(ts[len(ts) // 2], 3)
        outs.append(out.clone())
    row["equal"] = bool(torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2]))
    print(json.dumps(row), flush=True)
