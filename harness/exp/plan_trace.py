"""r4 probe: per-step host times of the 8-rank plan on one GPU (config 5, 2^30 keys through
labsort_sort_host_ranks with peer copies), from the LABSORT_PLAN_TRACE lines of the schedule
with harness/exp/plan_trace.patch applied (an experiment build; the product has no trace)."""
import importlib, os, sys
import numpy as np
REPO = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, REPO)
import torch
ls = importlib.import_module("radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd")
n = 1 << int(sys.argv[1] if len(sys.argv) > 1 else 30)
t = torch.empty(n, dtype=torch.int32, device="cuda:0")
ls.fill(t, n, 12345, "u31")
torch.cuda.synchronize()
src = t.cpu().numpy()
del t
torch.cuda.empty_cache()
work = np.empty_like(src)
for rep in range(3):
    np.copyto(work, src)
    print(f"--- rep {rep}", file=sys.stderr, flush=True)
    ls.sort_host_ranks(work, [0] * 8, transport="peer")
    ph, sent = ls.multi_timing()
    print(rep, {k: round(v, 3) for k, v in ph.items()}, flush=True)
