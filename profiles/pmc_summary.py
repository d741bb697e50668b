"""profiles/pmc_summary.py -- condense rocprofv3 output into committed summaries.

    python profiles/pmc_summary.py <gpurun_out dir> <tag> [--n 268435456]

Reads  <dir>/prof_<tag>/run_kernel_stats.csv           (--kernel-trace --stats pass)
       <dir>/pmc_FETCH_SIZE_<tag>/run_counter_collection.csv   (separate --pmc pass)
       <dir>/pmc_WRITE_SIZE_<tag>/run_counter_collection.csv   (separate --pmc pass)
Writes profiles/<tag>_kernel_stats.csv (copy of the stats summary) and
       profiles/<tag>_pmc.json: per labsort kernel class, average FETCH_SIZE and
       WRITE_SIZE per launch and the corrected HBM bytes per launch.

Correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced
streaming read, so read bytes = 2 x FETCH_SIZE x 1024; WRITE_SIZE is exact for
16-B streaming stores (our scatter stores are 4 B per lane: uncalibrated, so
the write side is reported as measured).  Infinity-Cache hits are counted.
"""
import csv
import json
import os
import shutil
import sys

CLASSES = {"k_onesweep": "onesweep", "k_histogram": "histogram", "k_hist_seg": "histogram",
           "k_km_blocks": "kmerge_blocks", "k_merge_pass": "merge",
           "k_tile_sort": "tile_sort", "k_merge_part": "partition", "k_merge_ab": "merge_ab",
           "k_count_descents": "count_descents", "k_fill": "fill", "k_final_copy": "final_copy",
           "k_wave_split": "wave_split", "k_gsweep": "gsweep", "k_gcopy": "gcopy"}


def klass(name):
    for k, v in CLASSES.items():
        if k in name:
            return v
    return None


def read_pmc(path, counter):
    acc = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            c = klass(row["Kernel_Name"])
            if c is None:
                continue
            a = acc.setdefault(c, [0.0, 0])
            a[0] += float(row["Counter_Value"])
            a[1] += 1
    return {c: v[0] / v[1] for c, v in acc.items() if v[1]}


def main():
    d, tag = sys.argv[1], sys.argv[2]
    n = int(sys.argv[sys.argv.index("--n") + 1]) if "--n" in sys.argv else 1 << 28
    here = os.path.dirname(os.path.abspath(__file__))
    stats = os.path.join(d, f"prof_{tag}", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(here, f"{tag}_kernel_stats.csv"))
    fetch = read_pmc(os.path.join(d, f"pmc_FETCH_SIZE_{tag}", "run_counter_collection.csv"), "FETCH_SIZE")
    write = read_pmc(os.path.join(d, f"pmc_WRITE_SIZE_{tag}", "run_counter_collection.csv"), "WRITE_SIZE")
    out = {"tag": tag, "n": n, "units": "bytes per launch",
           "correction": "read = 2 x FETCH_SIZE KiB (gfx950 half-count), write = WRITE_SIZE KiB as measured",
           "kernels": {}}
    for c in sorted(set(fetch) | set(write)):
        f, w = fetch.get(c, 0.0), write.get(c, 0.0)
        out["kernels"][c] = {"fetch_size_kib": round(f, 1), "write_size_kib": round(w, 1),
                             "read_bytes": 2 * f * 1024, "write_bytes": w * 1024,
                             "hbm_bytes_per_launch": 2 * f * 1024 + w * 1024,
                             "algorithmic_bytes_per_launch": {"onesweep": 8 * n, "histogram": 4 * n,
                                                              "merge": 8 * n, "tile_sort": 8 * n}.get(c)}
    with open(os.path.join(here, f"{tag}_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["kernels"].get("onesweep"), indent=1))


if __name__ == "__main__":
    main()
