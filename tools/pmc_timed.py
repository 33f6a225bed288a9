"""PMC counters of the TIMED launches of the driver's bench protocol, per x point.

Usage: python tools/pmc_timed.py <gpurun_out/tag> <profiles/tag> [steps] [x_points]

Reads the rocprofv3 runs of tools/profile_r04.sh -- every pass is the driver's command
`bench.py --gpus 1 --steps K --warmup W` (with --no-cpu --spot 0 --trajectory 0, so nothing
runs after the timed steps) -- and keeps, per pass, the dispatches of the K timed steps: a step
ends with its one cut_argmax2_kernel launch, so the last K of those delimit the timed steps;
inside a step the MAIN LP launch is the lp_hyper_kernel dispatch with the most fetched bytes
(the others are the refresh's training solves and the representatives' re-solve), the selection
kernels likewise.  Per kernel and x point (step i is at x point i % X): mean counter values per
launch, with the gfx950 FETCH_SIZE correction of MI355X_MICROARCH.md (x 2 for wide streaming
reads; reported next to the raw value, the LP's 4-8 B gathers are uncalibrated).  The bench
JSON line each pass printed (`*_bench.json`) gives the same steps' pivots and eta-arena
entries, so WRITE_SIZE of the main launch is split into the eta-file stores (12 B per entry)
and the rest by a least-squares fit over the timed steps.
"""
import csv
import glob
import gzip
import json
import os
import sys
from collections import defaultdict

import numpy as np

KERNELS = ["lp_hyper_kernel", "pool_refine_kernel", "pool_select_kernel", "cut_argmax2_kernel"]


def short(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


def load_pass(path):
    """dispatch id -> {name, counters, ms} (raw counter_collection.csv or prof_reduce.py's .csv.gz)"""
    disp = {}
    f = gzip.open(path, "rt", newline="") if path.endswith(".gz") else open(path, newline="")
    for r in csv.DictReader(f):
        d = int(r["Dispatch_Id"])
        e = disp.setdefault(d, {"name": r["Kernel_Name"], "c": {}, "ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6,
                                "scratch": int(float(r["Scratch_Size"])), "vgpr": int(float(r["VGPR_Count"]))})
        e["c"][r["Counter_Name"]] = e["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return disp


def timed_steps(disp, K):
    """per timed step: {kernel: the dispatch (largest FETCH/any counter) of that kernel in the step}"""
    ids = sorted(disp)
    cuts = [i for i in ids if "cut_argmax2_kernel" in disp[i]["name"]]
    if len(cuts) < K + 1:
        return []
    steps = []
    for a, b in zip(cuts[-K - 1:-1], cuts[-K:]):
        sel = {}
        for i in ids:
            if a < i <= b:
                k = short(disp[i]["name"])
                if not k:
                    continue
                val = sum(disp[i]["c"].values())
                if k not in sel or val > sum(disp[sel[k]]["c"].values()):
                    sel[k] = i
        steps.append({k: disp[i] for k, i in sel.items()})
    return steps


def main():
    src, dst = sys.argv[1], sys.argv[2]
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    X = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    os.makedirs(dst, exist_ok=True)
    per = defaultdict(lambda: defaultdict(lambda: defaultdict(list)))   # kernel -> x -> counter -> values
    meta = {}
    bench_lines = {}
    passes = {}
    for pdir in glob.glob(os.path.join(src, "pmc_*")):
        if os.path.isdir(pdir):
            fs = glob.glob(os.path.join(pdir, "**", "*counter_collection.csv"), recursive=True)
            if fs:
                passes[os.path.basename(pdir)] = fs[0]
        elif pdir.endswith("_counters.csv.gz"):
            passes[os.path.basename(pdir)[:-len("_counters.csv.gz")]] = pdir
    for tag, path in sorted(passes.items()):
        fs = [path]
        disp = load_pass(fs[0])
        steps = timed_steps(disp, K)
        for i, st in enumerate(steps):
            for k, d in st.items():
                for cn, v in d["c"].items():
                    per[k][i % X][cn].append(v)
                per[k][i % X]["profiled_ms_" + tag].append(d["ms"])
                meta[k] = {"scratch_bytes_per_lane": d["scratch"], "vgpr": d["vgpr"]}
        bj = os.path.join(src, f"{tag}_bench.json")
        if os.path.exists(bj):
            lines = [l for l in open(bj) if l.startswith("{")]
            if lines:
                bench_lines[tag] = json.loads(lines[-1])
    out = {"protocol": f"driver command bench.py --gpus 1 --steps {K} --warmup 5 (--no-cpu --spot 0 --trajectory 0): "
                       f"the {K} timed steps of each PMC pass, step i at x point i % {X}",
           "units": "FETCH_SIZE / WRITE_SIZE: bytes per launch (rocprofv3 KiB x 1024); fetch_corrected = 2 x raw "
                    "(gfx950 wide-read calibration, MI355X_MICROARCH.md); SQ_*: per launch",
           "kernels": {}}
    for k, byx in per.items():
        ent = {"meta": meta.get(k, {}), "per_x": {}}
        allc = defaultdict(list)
        for x, cs in sorted(byx.items()):
            row = {}
            for cn, vs in cs.items():
                scale = 1024.0 if cn in ("FETCH_SIZE", "WRITE_SIZE") else 1.0
                row[cn] = float(np.mean(vs)) * scale
                allc[cn] += [v * scale for v in vs]
            if "FETCH_SIZE" in row:
                row["fetch_corrected"] = 2.0 * row["FETCH_SIZE"]
            ent["per_x"][str(x)] = row
        ent["mean"] = {cn: float(np.mean(vs)) for cn, vs in allc.items()}
        if "FETCH_SIZE" in ent["mean"]:
            ent["mean"]["fetch_corrected"] = 2.0 * ent["mean"]["FETCH_SIZE"]
        out["kernels"][k] = ent
    # WRITE_SIZE of the main LP launch vs its eta-arena stores (12 B per entry): per x point the
    # analytic eta bytes of the same pass's timed steps (bench JSON), and the fit
    # WRITE = a * scenarios + b * eta_bytes over the x points
    bw = bench_lines.get("pmc_write")
    lp = per.get("lp_hyper_kernel", {})
    if bw and lp:
        n = bw["config"]["scenarios"]
        xs, ws, eb = [], [], []
        for x, cs in sorted(lp.items()):
            if "WRITE_SIZE" not in cs:
                continue
            xp = bw["x_points"][x]
            if xp.get("lp_eta_entries") is None:
                continue
            xs.append(x)
            ws.append(float(np.mean(cs["WRITE_SIZE"])) * 1024.0)
            eb.append(12.0 * xp["lp_eta_entries"])
        if xs:
            A = np.stack([np.full(len(xs), n, dtype=float), np.array(eb)], axis=1)
            coef, *_ = np.linalg.lstsq(A, np.array(ws), rcond=None)
            out["lp_write_split"] = {
                "x_points": xs, "write_size_bytes": ws, "eta_store_bytes": eb,
                "fit": {"bytes_per_scenario": float(coef[0]), "write_bytes_per_eta_byte": float(coef[1])},
                "outputs_bytes_per_scenario": "obj 8 + status 4 + iters 4 + ops 8 + etan 4 + pool pick 4 + dual key 8 = 40",
                "note": "WRITE_SIZE of the main launch per x point against its eta-arena store bytes (12 B per entry, "
                        "counted by the kernel); eta stores are the only writes that grow with the pivots"}
    out["bench_lines"] = {t: {k: b.get(k) for k in ("value", "ms_per_step", "phases_ms_per_step", "lp_pivots_mean")}
                          for t, b in bench_lines.items()}
    with open(os.path.join(dst, "pmc_timed.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: v["mean"] for k, v in out["kernels"].items()}, indent=1))
    if "lp_write_split" in out:
        print(json.dumps(out["lp_write_split"], indent=1))


if __name__ == "__main__":
    main()
