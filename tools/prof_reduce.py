"""Shrink one rocprofv3 output directory to what tools/pmc_timed.py reads (run on the GPU box
right after the pass, before the results travel back; the raw per-dispatch CSVs of a bench run
are larger than gpurun's copy-back limit).

Usage: python tools/prof_reduce.py <rocprofv3 -d dir> <out prefix>
Writes <out prefix>_counters.csv.gz (counter rows of this package's kernels: every kernel in the
twosd namespace), <out prefix>_trace.csv.gz (kernel-trace rows of the same kernels) and
<out prefix>_stats.csv (the --stats summary, all kernels) when the pass produced them; then
removes the directory.
"""
import csv
import glob
import gzip
import os
import shutil
import sys

KEEP_COLS = ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp",
             "Scratch_Size", "VGPR_Count", "LDS_Block_Size", "Grid_Size", "Workgroup_Size"]


def ours(name):
    return "twosd" in name


def reduce_csv(src, dst, cols=None):
    with open(src, newline="") as f, gzip.open(dst, "wt", newline="") as g:
        r = csv.DictReader(f)
        keep = [c for c in r.fieldnames if cols is None or c in cols]
        w = csv.DictWriter(g, fieldnames=keep, extrasaction="ignore")
        w.writeheader()
        n = 0
        for row in r:
            if ours(row.get("Kernel_Name", "")):
                w.writerow(row)
                n += 1
    return n


def main():
    src, pre = sys.argv[1], sys.argv[2]
    found = {}
    for p in glob.glob(os.path.join(src, "**", "*.csv"), recursive=True):
        b = os.path.basename(p)
        if b.endswith("counter_collection.csv"):
            found["counters"] = reduce_csv(p, pre + "_counters.csv.gz", KEEP_COLS)
        elif b.endswith("kernel_trace.csv"):
            found["trace"] = reduce_csv(p, pre + "_trace.csv.gz")
        elif b.endswith("kernel_stats.csv"):
            shutil.copy(p, pre + "_stats.csv")
            found["stats"] = 1
    shutil.rmtree(src, ignore_errors=True)
    print("reduced", src, found)


if __name__ == "__main__":
    main()
