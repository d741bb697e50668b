"""profiles/pmc_summary.py -- condense rocprofv3 output into committed summaries.

    python profiles/pmc_summary.py <gpurun_out dir> <tag> [--n 268435456]

Reads  <dir>/prof_<tag>/run_kernel_stats.csv           (--kernel-trace --stats pass)
       <dir>/pmc_FETCH_SIZE_<tag>/run_counter_collection.csv   (separate --pmc pass)
       <dir>/pmc_WRITE_SIZE_<tag>/run_counter_collection.csv   (separate --pmc pass)
       <dir>/cal_FETCH_SIZE_<tag>/run_counter_collection.csv   (harness/bin/pmc_cal, optional)
       <dir>/cal_WRITE_SIZE_<tag>/run_counter_collection.csv
Writes profiles/<tag>_kernel_stats.csv (copy of the stats summary) and
       profiles/<tag>_pmc.json: per labsort kernel class, average FETCH_SIZE and
       WRITE_SIZE per launch and the corrected HBM bytes per launch.

Correction.  FETCH_SIZE and WRITE_SIZE are in KiB.  MI355X_MICROARCH.md §HBM calibrates
only the 16-B/lane streaming read (FETCH_SIZE = 1/2 of the bytes); the labsort kernels
use 4-B/lane loads and stores, so harness/exp/pmc_cal.hip moves a known 1 GiB with each
access shape the product uses and this script derives a factor per shape
(bytes / counter bytes).  Each product kernel class is corrected by the factors of its
own load and store shapes (SHAPES); without a calibration pass the guide's x2 read /
x1 write rule is used and the summary says so.  Infinity-Cache hits are counted.
"""
import csv
import json
import os
import shutil
import sys

CLASSES = {"k_onesweep_p<true>": "onesweep_kv", "k_m4_merge_kv": "merge4_kv", "k_tile_sort<1024, 16, true>": "tile_sort_kv",
           "k_onesweep": "onesweep", "k_histogram": "histogram", "k_hist_seg": "histogram",
           "k_km_blocks": "kmerge_blocks", "k_merge_pass": "merge",
           "k_tile_sort": "tile_sort", "k_merge_part": "partition", "k_merge_ab": "merge_ab",
           "k_count_descents": "count_descents", "k_fill": "fill", "k_final_copy": "final_copy",
           "k_wave_split": "wave_split", "k_gsweep": "gsweep", "k_gcopy": "gcopy",
           "k_m4_merge": "merge4", "k_m4_rank": "merge4_rank"}


def klass(name):
    for k, v in CLASSES.items():
        if k in name:
            return v
    return None


def read_pmc(path, counter):
    """average counter value per launch and kernel class, over `path` and, if present, the
    merge-bench pass beside it (<dir>_merge)"""
    acc = {}
    paths = [path] + [p for p in [path.replace(os.sep + "run_counter", "_merge" + os.sep + "run_counter")]
                      if p != path and os.path.exists(p)]
    rows = [row for p in paths for row in csv.DictReader(open(p))
            if row["Counter_Name"] == counter and klass(row["Kernel_Name"]) is not None]
    # only each class's full-size launches: the bench's small legs (configs 1 and 2) launch
    # the same kernels on 2^16-2^20 keys, whose grids are a fraction of the 2^28 ones
    gmax = {}
    for row in rows:
        c = klass(row["Kernel_Name"])
        gmax[c] = max(gmax.get(c, 0), int(row["Grid_Size"]))
    for row in rows:
        c = klass(row["Kernel_Name"])
        if int(row["Grid_Size"]) * 2 < gmax[c]:
            continue
        a = acc.setdefault(c, [0.0, 0])
        a[0] += float(row["Counter_Value"])
        a[1] += 1
    return {c: v[0] / v[1] for c, v in acc.items() if v[1]}


# access shapes of each kernel class (the instructions in its ISA): read, write
SHAPES = {"onesweep": ("cal_rd_buf_nt", "cal_wr_buf"),      # buffer_load_dword nt / buffer_store_dword
          "onesweep_kv": ("cal_rd_buf_nt", "cal_wr_buf"),
          "histogram": ("cal_rd_x4_nt", None),                # global_load_dwordx4 nt (k_hist_seg)
          "merge": ("cal_rd_dword", "cal_wr_x4"),             # global_load_dword / global_store_dwordx4
          "tile_sort": ("cal_rd_dword", "cal_wr_dword"),      # global_load_dword / global_store_dword
          "merge4": ("cal_rd_dword", "cal_wr_x4"),            # global_load_dword nt / global_store_dwordx4 nt
          "merge4_kv": ("cal_rd_dword", "cal_wr_x4"),
          "tile_sort_kv": ("cal_rd_dword", "cal_wr_dword"),
          "count_descents": ("cal_rd_dword", None),           # global_load_dword (a check: 1 GiB read)
          "fill": (None, "cal_wr_dword")}                     # global_store_dword (a check: 1 GiB written)
CAL_BYTES = float(1 << 30)  # every calibration kernel moves 2^28 words per launch


def calibration(d, tag):
    """{shape: bytes per counter byte} from the pmc_cal passes, or None"""
    f = os.path.join(d, f"cal_FETCH_SIZE_{tag}", "run_counter_collection.csv")
    w = os.path.join(d, f"cal_WRITE_SIZE_{tag}", "run_counter_collection.csv")
    if not (os.path.exists(f) and os.path.exists(w)):
        return None

    def per_kernel(path, counter):
        acc = {}
        for row in csv.DictReader(open(path)):
            if row["Counter_Name"] != counter or not row["Kernel_Name"].startswith("cal_"):
                continue
            k = row["Kernel_Name"].split("(")[0]
            a = acc.setdefault(k, [0.0, 0])
            a[0] += float(row["Counter_Value"])
            a[1] += 1
        return {k: v[0] / v[1] for k, v in acc.items()}

    fetch, write = per_kernel(f, "FETCH_SIZE"), per_kernel(w, "WRITE_SIZE")
    cal = {}
    for k, kib in fetch.items():
        if k.startswith("cal_rd") and kib > 0:
            cal[k] = {"counter_kib": round(kib, 1), "factor": CAL_BYTES / (kib * 1024)}
    for k, kib in write.items():
        if k.startswith("cal_wr") and kib > 0:
            cal[k] = {"counter_kib": round(kib, 1), "factor": CAL_BYTES / (kib * 1024)}
    return cal


def main():
    d, tag = sys.argv[1], sys.argv[2]
    n = int(sys.argv[sys.argv.index("--n") + 1]) if "--n" in sys.argv else 1 << 28
    here = os.path.dirname(os.path.abspath(__file__))
    for leg in ("", "_merge"):
        stats = os.path.join(d, f"prof_{tag}{leg}", "run_kernel_stats.csv")
        if os.path.exists(stats):
            shutil.copy(stats, os.path.join(here, f"{tag}{leg}_kernel_stats.csv"))
    fetch = read_pmc(os.path.join(d, f"pmc_FETCH_SIZE_{tag}", "run_counter_collection.csv"), "FETCH_SIZE")
    write = read_pmc(os.path.join(d, f"pmc_WRITE_SIZE_{tag}", "run_counter_collection.csv"), "WRITE_SIZE")
    cal = calibration(d, tag)
    out = {"tag": tag, "n": n, "units": "bytes per launch",
           "correction": ("per access shape from harness/exp/pmc_cal.hip (calibration below): read = FETCH_SIZE "
                          "x factor(read shape), write = WRITE_SIZE x factor(write shape)") if cal else
                         "read = 2 x FETCH_SIZE KiB (gfx950 half-count, 16-B reads), write = WRITE_SIZE KiB as measured "
                         "(uncalibrated)",
           "calibration": cal, "kernels": {}}
    for c in sorted(set(fetch) | set(write)):
        f, w = fetch.get(c, 0.0), write.get(c, 0.0)
        rs, ws = SHAPES.get(c, (None, None))
        fr = cal[rs]["factor"] if cal and rs in cal else 2.0
        fw = cal[ws]["factor"] if cal and ws in cal else 1.0
        out["kernels"][c] = {"fetch_size_kib": round(f, 1), "write_size_kib": round(w, 1),
                             "read_shape": rs, "write_shape": ws, "read_factor": round(fr, 4),
                             "write_factor": round(fw, 4),
                             "read_bytes": fr * f * 1024, "write_bytes": fw * w * 1024,
                             "hbm_bytes_per_launch": fr * f * 1024 + fw * w * 1024,
                             "algorithmic_bytes_per_launch": {"onesweep": 8 * n, "onesweep_kv": 16 * n, "histogram": 4 * n,
                                                              "merge": 8 * n, "tile_sort": 8 * n, "merge4": 8 * n,
                                                              "merge4_kv": 16 * n, "tile_sort_kv": 16 * n,
                                                              "count_descents": 4 * n, "fill": 4 * n}.get(c)}
    with open(os.path.join(here, f"{tag}_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["kernels"].get("onesweep"), indent=1))


if __name__ == "__main__":
    main()
