"""Diagnostic (r4): run the keys-only 8-bit radix (local-pass path) on n keys and check
every intermediate the workspace still holds against numpy: the local pass's tile rows
and digit-0 totals, the run tables (ls, sr, first), the plan, and each launch's output
buffer that survives.  Usage: python lpath_debug.py N DIST [PARAM]"""
import importlib, os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, R)
import torch
ls = importlib.import_module("radix-sort-merge-sort-cuda---lab-y-practicos-gpgpu-2023_amd")

T, NSEG, GROUP, NCTR = 16384, 16, 64, 8
SIZEOF_PLAN, SIZEOF_SEGPLAN = 656, 16576


def up(x, a):
    return (x + a - 1) // a * a


def layout(n):
    ntp = (n + T - 1) // T
    ng = (ntp + GROUP - 1) // GROUP
    ntiles = ntp + NSEG
    o = 0
    L = {"ntp": ntp}
    L["err"] = o; o += 256
    L["tot0"] = o; o += 256 * 4
    L["joint"] = o; o += 4 * NSEG * 256 * 4
    L["counter"] = o; o += 3 * NCTR * 4
    L["gctr"] = o; o = up(o + 4, 256)
    L["flags"] = o; o = up(o + ng * 256 * 4, 256)
    L["lookback"] = o; o = up(o + 3 * ntiles * 256 * 4, 256)
    L["plan"] = o; o = up(o + SIZEOF_PLAN, 256)
    L["segplan"] = o; o = up(o + 3 * SIZEOF_SEGPLAN, 256)
    L["hist"] = o; o = up(o + 4 * 256 * 4, 256)
    L["rows"] = o; o = up(o + ntp * 256 * 4, 256)
    L["ls"] = o; o = up(o + (256 * ntp + 1) * 4, 256)
    L["sr"] = o; o = up(o + 256 * ntp * 4, 256)
    L["first"] = o; o = up(o + (ntp + 1) * 4, 256)
    L["tmp"] = up(o, 65536)
    L["tmp2"] = up(L["tmp"] + n * 4, 65536)
    return L


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32769
    dist = sys.argv[2] if len(sys.argv) > 2 else "u32"
    param = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    d = torch.empty(n, dtype=torch.int32, device="cuda")
    ls.fill(d, n, 0x5EED0003, dist, param)
    x = d.cpu().numpy().view(np.uint32).copy()
    o = torch.empty_like(d)
    wsb = ls.workspace_bytes(n, "radix")
    L = layout(n)
    assert wsb >= L["tmp2"] + n * 4, (wsb, L["tmp2"] + n * 4)
    ws = torch.full((wsb,), 0xAB, dtype=torch.uint8, device="cuda")
    o.fill_(-1)
    ls.sort_device(d, o, n, algo="radix", workspace=ws)
    torch.cuda.synchronize()
    W = ws.cpu().numpy()

    def u32(off, cnt):
        return W[off:off + 4 * cnt].view(np.uint32)

    ntp = L["ntp"]
    dg = [(x >> np.uint32(8 * p)) & np.uint32(255) for p in range(4)]
    print(f"n={n} dist={dist} ntp={ntp} err={u32(L['err'], 1)[0]}")
    # local pass: rows, totals
    rows = u32(L["rows"], ntp * 256).reshape(ntp, 256)
    bad = 0
    for t in range(ntp):
        c = np.bincount(dg[0][t * T:(t + 1) * T], minlength=256)
        ex = np.concatenate([[0], np.cumsum(c)[:-1]])
        bad += int(np.sum(rows[t] != (ex | (c << 16)).astype(np.uint32)))
    print("rows mismatches", bad)
    tot0 = u32(L["tot0"], 256)
    print("tot0 ok", bool(np.all(tot0 == np.bincount(dg[0], minlength=256))))
    # run tables
    cnt = np.stack([np.bincount(dg[0][t * T:(t + 1) * T], minlength=256) for t in range(ntp)])  # [t][d]
    runs = cnt.T.reshape(-1)  # e = d*ntp + t
    lsx = np.concatenate([[0], np.cumsum(runs)]).astype(np.uint32)
    lsg = u32(L["ls"], 256 * ntp + 1)
    print("ls mismatches", int(np.sum(lsg != lsx)), "first bad e", np.nonzero(lsg != lsx)[0][:8])
    loc = np.stack([np.concatenate([[0], np.cumsum(cnt[t])[:-1]]) for t in range(ntp)])
    srx = (np.arange(ntp)[None, :] * T + loc.T).reshape(-1).astype(np.uint32)
    srg = u32(L["sr"], 256 * ntp)
    nz = runs > 0
    print("sr mismatches (non-empty runs)", int(np.sum((srg != srx) & nz)))
    fx = np.zeros(ntp + 1, dtype=np.uint32)
    for k in range(ntp + 1):
        pos = min(k * T, n - 1) if k < ntp else n - 1
        fx[k] = np.searchsorted(lsx[1:], pos, side="right")
    fg = u32(L["first"], ntp + 1)
    print("first got", fg[:8], "expected", fx[:8], "ok", bool(np.all(fg == fx)))
    # joint fields: joint[(p+1)][nibble of digit p][digit p+1]
    jg = u32(L["joint"], 4 * NSEG * 256).reshape(4, NSEG, 256)
    for p in range(3):
        f = (x >> np.uint32(8 * p + 4)) & np.uint32(4095)
        jx = np.bincount((f & 15) * 256 + (f >> 4), minlength=NSEG * 256).reshape(NSEG, 256)
        print(f"joint[{p + 1}] mismatches", int(np.sum(jg[p + 1] != jx)))
    # launch 0's segment plan: starts by the top nibble of digit 0, bases per (segment, digit 1)
    sp = u32(L["segplan"], SIZEOF_SEGPLAN // 4)
    st = sp[0:17]
    nib0 = (dg[0] >> np.uint32(4)).astype(np.int64)
    stx = np.concatenate([[0], np.cumsum(np.bincount(nib0, minlength=16))]).astype(np.uint32)
    print("segplan0 start ok", bool(np.all(st == stx)), st[:6], stx[:6], "mode", sp[35], "segbits", sp[36], "maxt", sp[34])
    base = sp[48:48 + 4096].reshape(16, 256)
    j1 = np.bincount(nib0 * 256 + dg[1], minlength=4096).reshape(16, 256)
    g1 = np.concatenate([[0], np.cumsum(np.bincount(dg[1], minlength=256))[:-1]])
    bx = (g1[None, :] + np.concatenate([np.zeros((1, 256), np.int64), np.cumsum(j1, axis=0)[:-1]], axis=0)).astype(np.uint32)
    print("segplan0 base mismatches", int(np.sum(base != bx)))
    plan = u32(L["plan"], SIZEOF_PLAN // 4)
    print("plan src", plan[0:4], "dst", plan[32:36], "digit", plan[128:132], "copy_from", plan[160], "active", plan[161])
    # expected launch outputs
    order = np.argsort(dg[0], kind="stable")
    cur = x[order]
    outs = []
    for dig in [p for p in (1, 2, 3) if len(np.unique(dg[p])) > 1]:
        cur = cur[np.argsort((cur >> np.uint32(8 * dig)) & np.uint32(255), kind="stable")]
        outs.append((dig, cur.copy()))
    for j, (dig, e) in enumerate(outs):
        sel = plan[32 + j]
        name = {1: "OUT", 2: "tmp", 3: "tmp2"}.get(int(sel), str(sel))
        got = o.cpu().numpy().view(np.uint32) if name == "OUT" else (u32(L[name], n) if name in L else None)
        if got is None:
            print(f"launch {j} digit {dig} -> sel {sel}: ?")
            continue
        mism = np.nonzero(got != e)[0]
        print(f"  launch {j}: permutation of the input: {bool(np.array_equal(np.sort(got), np.sort(x)))}")
        if mism.size and j == 0:
            lo = order  # logical order: x[lo[i]] at logical position i
            inv = {int(v): i for i, v in enumerate(x[lo])} if n < (1 << 22) else {}
            for q in mism[:4]:
                g = int(got[q])
                print(f"  pos {q}: got {g:#010x} (logical pos {inv.get(g)}, digit1 {(g >> 8) & 255}, seg {(g >> 4) & 15}),"
                      f" expected {int(e[q]):#010x} (logical pos {inv.get(int(e[q]))}, seg {(int(e[q]) >> 4) & 15})")
        print(f"launch {j} digit {dig} -> {name}: mismatches {mism.size}", mism[:10], got[mism[:5]] if mism.size else "",
              e[mism[:5]] if mism.size else "")
    final = o.cpu().numpy().view(np.uint32)
    print("final sorted ok", bool(np.all(final == np.sort(x))))


main()
