"""Diagnostic: time the standalone digit histogram (labsort_histogram, old layout)
against the sort's segment-aligned histogram (first kernel of a radix sort) on the
same 2^28 uniform input."""
import importlib, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
ls = importlib.import_module("radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd")
n = 1 << 28
t = torch.empty(n, dtype=torch.int32, device="cuda")
ls.fill(t, n, 0x5EED0003, "u32")
h = torch.zeros(1024, dtype=torch.int32, device="cuda")
for _ in range(3):
    ls.histogram(t, n, h)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(10):
    ls.histogram(t, n, h)
b.record(); torch.cuda.synchronize()
print("labsort_histogram (k_histogram<8>) ms:", a.elapsed_time(b) / 10)
ls.timing_enable(True)
o = torch.empty_like(t)
for _ in range(10):
    ls.sort_device(t, o, n)
torch.cuda.synchronize()
print("sort's k_hist_seg ms:", ls.timing_read("histogram")[0] / ls.timing_read("histogram")[1])
