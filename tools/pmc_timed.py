"""PMC counters of the TIMED launches of the driver's bench protocol, per x point.

Usage: python tools/pmc_timed.py <gpurun_out/tag> <profiles/tag> [steps] [x_points]
(steps, x points and epigraphs are taken from the passes' own bench JSON lines when present; the
summary carries the workload key bench.py matches on -- pmc_summary.json for the storm driver
workload, pmc_summary_<instance>_<N>_V<|V|>_E<E>.json for any other)

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

KERNELS = ["lp_hyper_kernel", "pool_refine_kernel", "pool_select_kernel", "cut_argmax3_kernel", "cut_argmax2_kernel",
           "cut_fixup_kernel", "pg_ftran_kernel", "pg_fill_kernel"]


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


def load_trace(path):
    """dispatch id -> {name, ms} of a kernel-trace CSV (prof_reduce.py's .csv.gz or raw)"""
    disp = {}
    f = gzip.open(path, "rt", newline="") if path.endswith(".gz") else open(path, newline="")
    for r in csv.DictReader(f):
        disp[int(r["Dispatch_Id"])] = {"name": r["Kernel_Name"], "c": {},
                                       "ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6}
    return disp


def timed_steps(disp, K):
    """per timed step: {kernel: the dispatch (largest FETCH/any counter; by duration in a trace) of
    that kernel in the step}"""
    ids = sorted(disp)
    # one cut per sub-step: its argmax launch (the fp32 pass, or the fp64 one; a cut launches both
    # and the idle one returns at once, so the step boundary is the fp64 kernel, launched last)
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
                val = sum(disp[i]["c"].values()) or disp[i]["ms"]
                if k not in sel or val > (sum(disp[sel[k]]["c"].values()) or disp[sel[k]]["ms"]):
                    sel[k] = i
        steps.append({k: disp[i] for k, i in sel.items()})
    return steps


def bench_config(src):
    """(steps, warmup, x points, epigraphs, key) of the bench command the passes ran, from the JSON line
    of any pass (every pass runs the same command)"""
    for bj in sorted(glob.glob(os.path.join(src, "*_bench.json"))):
        lines = [l for l in open(bj) if l.startswith("{")]
        if lines:
            d = json.loads(lines[-1])
            c = d["config"]
            key = {"instance": c["instance"], "scenarios": c["scenarios"], "vertices": c["vertices"],
                   "epigraphs": c["epigraphs"], "n_gpus": d["n_gpus"]}
            return d["steps"], d["warmup"], c["x_points"], c["epigraphs"], key, c["workload"]
    return None


def main():
    src, dst = sys.argv[1], sys.argv[2]
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    X = int(sys.argv[4]) if len(sys.argv) > 4 else 4
    E, key, W, workload = 1, None, 5, None
    cfg = bench_config(src)
    if cfg:   # the command's own steps / x points / epigraphs and the workload key
        K, W, X, E, key, workload = cfg
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
        # one cut launch per epigraph and step: every epigraph's pass is a sub-step
        steps = timed_steps(disp, K * E)
        for i, st in enumerate(steps):
            xi = (i // E) % X
            for k, d in st.items():
                for cn, v in d["c"].items():
                    per[k][xi][cn].append(v)
                per[k][xi]["profiled_ms_" + tag].append(d["ms"])
                meta[k] = {"scratch_bytes_per_lane": d["scratch"], "vgpr": d["vgpr"]}
        bj = os.path.join(src, f"{tag}_bench.json")
        if os.path.exists(bj):
            lines = [l for l in open(bj) if l.startswith("{")]
            if lines:
                bench_lines[tag] = json.loads(lines[-1])
    out = {"protocol": f"bench.py --gpus 1 --steps {K} --warmup {W} (--no-cpu --spot 0 --trajectory 0): "
                       f"the {K} timed steps of each PMC pass ({E} epigraph pass(es) each), step i at x point i % {X}",
           "key": key, "workload": workload,
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
    if bw and lp and E == 1:
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
    # timed-step kernel durations from the trace pass (no counters: undisturbed timing)
    dur = defaultdict(list)
    tr = glob.glob(os.path.join(src, "trace_trace.csv.gz")) + glob.glob(os.path.join(src, "trace", "**", "*kernel_trace.csv"), recursive=True)
    if tr:
        for st in timed_steps(load_trace(tr[0]), K * E):
            for k, d in st.items():
                dur[k].append(d["ms"])
    out["trace_ms"] = {k: float(np.mean(v)) for k, v in dur.items()}
    kk = key or {"instance": "storm", "scenarios": 1_000_000, "vertices": 4096, "epigraphs": 1}
    is_default = (kk["instance"], kk["scenarios"], kk["vertices"], kk["epigraphs"]) == ("storm", 1_000_000, 4096, 1)
    suffix = "" if is_default else f"_{kk['instance']}_{kk['scenarios']}_V{kk['vertices']}_E{kk['epigraphs']}"
    with open(os.path.join(dst, f"pmc_timed{suffix}.json"), "w") as f:
        json.dump(out, f, indent=1)
    # the summary bench.py reads (latest profiles/r*/pmc_summary.json): per kernel, the mean over
    # the timed launches of the driver's protocol
    summ = {"workload": (workload or "storm 1000000 scenarios") + f"; bench.py --gpus 1 --steps {K} --warmup {W}, 1 MI355X",
            "key": key or {"instance": "storm", "scenarios": 1_000_000, "vertices": 4096, "epigraphs": 1, "n_gpus": 1},
            "source": "rocprofv3 --kernel-trace --stats and separate --pmc passes over that command "
                      "(tools/profile_r04.sh, reduced on the box by tools/prof_reduce.py); means over the timed steps' "
                      "launches (tools/pmc_timed.py)",
            "correction": "FETCH_SIZE/WRITE_SIZE are KiB; hbm_bytes = 1024*(2*FETCH_SIZE + WRITE_SIZE) (the guide's gfx950 "
                          "correction for wide reads; an upper estimate for narrow accesses); hbm_bytes_raw = "
                          "1024*(FETCH_SIZE + WRITE_SIZE)",
            "scenarios": (key or {}).get("scenarios", 1_000_000), "kernels": {}}
    for k, ent in out["kernels"].items():
        m = ent["mean"]
        f_kib = m.get("FETCH_SIZE", 0.0) / 1024.0
        w_kib = m.get("WRITE_SIZE", 0.0) / 1024.0
        ms = out["trace_ms"].get(k)
        e = {"duration_ms": ms, "FETCH_SIZE_KiB": f_kib, "WRITE_SIZE_KiB": w_kib,
             "hbm_bytes_per_launch": 1024.0 * (2 * f_kib + w_kib), "hbm_bytes_per_launch_raw": 1024.0 * (f_kib + w_kib),
             "scratch_bytes_per_lane": ent["meta"].get("scratch_bytes_per_lane")}
        for cn in ("SQ_INSTS_VALU_MFMA_MOPS_F64", "SQ_INSTS_VALU_MFMA_F64", "SQ_INSTS_VALU_MFMA_MOPS_F32", "SQ_INSTS_VALU_MFMA_F32",
                   "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES",
                   "GRBM_GUI_ACTIVE", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
                   "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA"):
            if cn in m:
                e[cn] = m[cn]
        f32 = bool(m.get("SQ_INSTS_VALU_MFMA_MOPS_F32"))
        mops = m.get("SQ_INSTS_VALU_MFMA_MOPS_F32") if f32 else m.get("SQ_INSTS_VALU_MFMA_MOPS_F64")
        if ms and mops:
            fl = 512.0 * mops
            tag = "f32" if f32 else "f64"
            e[f"mfma_{tag}_flops"] = fl
            e[f"mfma_{tag}_tflops_counted"] = fl / (ms * 1e-3) / 1e12
            e["mfma_util"] = e[f"mfma_{tag}_tflops_counted"] / (157.3 if f32 else 78.6)
            if m.get("GRBM_GUI_ACTIVE"):
                e["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8.0 * 1024.0)
        summ["kernels"][k] = e
    if "lp_write_split" in out:
        summ["lp_write_split"] = out["lp_write_split"]["fit"]
    with open(os.path.join(dst, f"pmc_summary{suffix}.json"), "w") as f:
        json.dump(summ, f, indent=1)
    print(json.dumps({k: v["mean"] for k, v in out["kernels"].items()}, indent=1))
    if "lp_write_split" in out:
        print(json.dumps(out["lp_write_split"], indent=1))


if __name__ == "__main__":
    main()
