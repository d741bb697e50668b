"""labsort_sort_device is a fixed, allocation-free sequence of launches and memsets on
the caller's stream (include/labsort.h), so it can be captured in a HIP graph and
replayed: captured through torch.cuda.graph for every algorithm, replayed on new input
data written into the same buffers, and checked against std::sort (the oracle)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("algo,impl,n", [("radix", "gather", (1 << 20) + 5), ("radix", "onesweep", (1 << 20) + 5),
                                         ("radix", "onesweep", 1 << 26), ("merge", "", 3 * (1 << 20) + 1),
                                         ("radix1", "", 100_003)])
def test_sort_device_graph_replay(ls, oracle, torch_gpu, monkeypatch, algo, impl, n):
    torch = torch_gpu
    if impl:
        monkeypatch.setenv("LABSORT_RADIX_IMPL", impl)
    src = torch.empty(n, dtype=torch.int32, device="cuda")
    out = torch.empty_like(src)
    ws = torch.empty(max(ls.workspace_bytes(n, algo), 256), dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    ls.fill(src, n, 0x5EEDA000, "u32", stream=s)
    with torch.cuda.stream(s):  # warm-up outside the capture
        ls.sort_device(src, out, n, algo=algo, workspace=ws, stream=s)
    s.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        ls.sort_device(src, out, n, algo=algo, workspace=ws, stream=torch.cuda.current_stream())
    for seed in (0x5EEDA001, 0x5EEDA002):
        ls.fill(src, n, seed, "mod1000" if seed & 1 else "u32")
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        ls.workspace_status(ws, n, algo)
        exp = oracle.sort_u32(oracle.gen(n, seed, "mod1000" if seed & 1 else "u32"))
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), exp)
