"""Summarise one profile_round.sh run into profiles/<tag>/pmc_summary.json.

Usage: python tools/pmc_summarize.py <gpurun_out/tag> <profiles/tag> <scenarios>

Reads the rocprofv3 kernel trace (trace/run_kernel_trace.csv, stats copied alongside) and
the two separate PMC passes (pmc_fetch, pmc_write: FETCH_SIZE / WRITE_SIZE in KiB per
dispatch) and writes, per kernel of the hot path, for its LARGEST dispatch (the full
1M-scenario launch; setup launches such as the pool build and the |V| pool are smaller):
duration, PMC bytes per launch (the gfx950 correction
of MI355X_MICROARCH.md: hbm_bytes = 1024 * (2 * FETCH_SIZE + WRITE_SIZE), an upper
estimate for narrow accesses), scratch bytes per lane.  Also copies the CSVs it used.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

KERNELS = ["lp_hyper_kernel", "pool_select_kernel", "pool_refine_kernel", "pool_selstream_kernel", "pool_xbase_kernel", "cut_argmax2_kernel", "cut_argmax_kernel", "cut_fixup_kernel", "cut_vbase_kernel",
           "cut_pk_kernel", "cut_pktc_kernel", "vkey_insert_kernel", "dvs_batch_kernel", "dvs_lookup_kernel", "dvs_assign_kernel"]


def short(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


def main():
    src, dst, scen = sys.argv[1], sys.argv[2], int(sys.argv[3])
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    dur = {}
    if stats:
        shutil.copy(stats[0], os.path.join(dst, "kernel_stats.csv"))
    traces = glob.glob(os.path.join(src, "trace", "**", "*kernel_trace.csv"), recursive=True)
    if traces:
        for r in csv.DictReader(open(traces[0])):
            k = short(r["Kernel_Name"])
            if k:
                d = (float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e6
                dur[k] = max(dur.get(k, 0.0), d)
    # timed-region stats: the trace run is bench.py --steps K --warmup 1 --spot 0 (K = 4 by
    # default), one cut_argmax_kernel launch per step, so the timed steps start after the
    # (K+1)-th last of those (the warmup's) and the cut kernels trailing it; per kernel:
    # launches, average and total duration inside that region (what the bench's events time)
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    if traces:
        rows = sorted(csv.DictReader(open(traces[0])), key=lambda r: int(r["Start_Timestamp"]))
        cuts = [i for i, r in enumerate(rows) if "cut_argmax" in r["Kernel_Name"]]
        if len(cuts) >= steps + 1:
            i0 = cuts[-steps - 1] + 1
            while i0 < len(rows) and "cut_" in rows[i0]["Kernel_Name"]:
                i0 += 1
            agg = defaultdict(list)
            for r in rows[i0:]:
                agg[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
            with open(os.path.join(dst, "timed_kernel_stats.csv"), "w", newline="") as fh:
                wr = csv.writer(fh)
                wr.writerow(["Name", "Calls", "AverageMs", "TotalMs", "MinMs", "MaxMs"])
                for name, ds in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
                    wr.writerow([name, len(ds), round(sum(ds) / len(ds), 6), round(sum(ds), 6), round(min(ds), 6),
                                 round(max(ds), 6)])
    pmc = defaultdict(lambda: defaultdict(list))
    scratch = {}
    for tag in ("pmc_fetch", "pmc_write", "pmc_mfma"):
        fs = glob.glob(os.path.join(src, tag, "**", "*counter_collection.csv"), recursive=True)
        if not fs:
            continue
        shutil.copy(fs[0], os.path.join(dst, f"{tag}.csv"))
        for r in csv.DictReader(open(fs[0])):
            k = short(r["Kernel_Name"])
            if k:
                pmc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                scratch[k] = int(float(r["Scratch_Size"]))
    out = {"workload": f"storm {scen} scenarios, bench.py defaults, 1 MI355X",
           "source": "rocprofv3 --kernel-trace --stats; separate --pmc FETCH_SIZE / --pmc WRITE_SIZE / fp64 MFMA passes "
                     "(tools/profile_round.sh)",
           "correction": "FETCH_SIZE/WRITE_SIZE are KiB; gfx950 FETCH_SIZE counts 1/2 of wide coalesced (16 B/lane) reads, "
                         "so hbm_bytes = 1024*(2*FETCH_SIZE + WRITE_SIZE) (the guide's correction; an upper estimate for "
                         "narrow accesses); hbm_bytes_raw = 1024*(FETCH_SIZE + WRITE_SIZE) is the estimate for kernels "
                         "whose reads are 8 B per lane (the cut kernel's delta loads)",
           "scenarios": scen, "kernels": {}}
    for k in KERNELS:
        c = pmc.get(k)
        if not c and k not in dur:
            continue
        e = {"duration_ms": dur.get(k)}
        if c:
            f = max(c.get("FETCH_SIZE", [0.0]))
            w = max(c.get("WRITE_SIZE", [0.0]))
            e.update({"FETCH_SIZE_KiB": f, "WRITE_SIZE_KiB": w, "hbm_bytes_per_launch": 1024.0 * (2 * f + w),
                      "hbm_bytes_per_launch_raw": 1024.0 * (f + w),
                      "scratch_bytes_per_lane": scratch.get(k)})
        if c and "SQ_INSTS_VALU_MFMA_MOPS_F64" in c:
            mops = max(c["SQ_INSTS_VALU_MFMA_MOPS_F64"])
            busy = max(c.get("SQ_VALU_MFMA_BUSY_CYCLES", [0.0]))
            gui = max(c.get("GRBM_GUI_ACTIVE", [0.0]))
            e.update({"SQ_INSTS_VALU_MFMA_MOPS_F64": mops, "SQ_INSTS_VALU_MFMA_F64": max(c.get("SQ_INSTS_VALU_MFMA_F64", [0.0])),
                      "SQ_VALU_MFMA_BUSY_CYCLES": busy, "SQ_BUSY_CYCLES": max(c.get("SQ_BUSY_CYCLES", [0.0])),
                      "GRBM_GUI_ACTIVE": gui, "mfma_f64_flops": 512.0 * mops})
            if dur.get(k):
                e["mfma_f64_tflops_counted"] = 512.0 * mops / (dur[k] * 1e-3) / 1e12
                e["mfma_util"] = e["mfma_f64_tflops_counted"] / 78.6   # counted MFMA flops / kernel time vs the fp64 spec
            if gui > 0:
                e["mfma_busy_frac"] = busy / (gui * 4.0 * 256.0 / 8.0)   # per-SIMD busy cycles / (GRBM cycles (8 XCDs) x SIMDs)
        out["kernels"][k] = e
    with open(os.path.join(dst, "pmc_summary.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
