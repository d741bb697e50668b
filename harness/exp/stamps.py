"""Diagnostic: per-phase cycles of the onesweep tile loop (build: harness/exp/build_stamps.sh).
Sorts 2^28 uniform keys a few times and prints each phase's share of the wave time."""
import ctypes, importlib, os, sys
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
lib = os.environ.setdefault("LABSORT_LIBRARY", os.path.join(R, "harness/exp/liblabsort_stamps.so"))
import torch
ls = importlib.import_module("radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd")
L = ctypes.CDLL(lib)
buf = (ctypes.c_ulonglong * 16)()
n = 1 << int(os.environ.get("LOG2N", "28"))
t = torch.empty(n, dtype=torch.int32, device="cuda")
ls.fill(t, n, 0x5EED0003, "u32")
o = torch.empty_like(t)
for _ in range(2):
    ls.sort_device(t, o, n)
torch.cuda.synchronize()
L.labsort_exp_stamps(buf, 1)
steps = 5
for _ in range(steps):
    ls.sort_device(t, o, n)
torch.cuda.synchronize()
L.labsort_exp_stamps(buf, 1)
names = ["look-back issue + B load wait", "rank B", "look-back completion A", "barrier 2",
         "aggregate B + scatter A issue", "barrier 2b", "offsets + acquire", "barrier 3",
         "reorder + barrier 4", "readback + joint"]
tot = sum(buf[i] for i in range(10))
blocks = buf[10]
print(f"blocks {blocks}, total wave-cycles {tot:.3e}, per block-launch per wave {tot / blocks / 16:.0f}")
for i, nm in enumerate(names):
    print(f"{nm:32s} {100 * buf[i] / tot:6.1f} %  {buf[i] / blocks / 16:10.0f} cycles/wave/launch")
print(f"look-backs {buf[14]}, extra rounds per look-back {buf[11] / max(buf[14], 1):.2f}, "
      f"stalled rounds {buf[12] / max(buf[14], 1):.2f}, tiles walked {buf[13] / max(buf[14], 1):.2f}")
