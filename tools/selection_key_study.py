"""Offline study of warm-start selection keys (CPU, development).  Reads
the per-(pool basis, scenario) pivot tables tools/ssn_hindsight.py dumps on the GPU box
(HINDSIGHT_DUMP=gpurun_out/hs ... storm -> gpurun_out/hs_storm_x<i>.npz: oracle pivots from every
pool basis, the pool heads, the sample's values and x), forms x_B = B_p^-1 b_s of every basis and
scenario with numpy, and reports the mean pivots a flat search over the whole pool would reach
with each candidate key (argmin over the bases), next to the device's picks and the hindsight floor.
Usage: python tools/selection_key_study.py   (after copying the dumps to gpurun_out/)"""
import numpy as np, sys, time
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from tests import instances as I
import scipy.linalg as sl
inst = I.load("storm"); sp = inst["osp2"]
W = np.asarray(sp.W, dtype=float); m, n = W.shape
sense = np.array([s if isinstance(s, str) else chr(s) for s in sp.senses])
taus = [1e-6, 1e-2, 1, 10, 100, 1000]
for tag in ["x0", "x4"]:
    z = np.load(f"gpurun_out/hs_storm_{tag}.npz")
    allit, heads, picks, vals, x, rows = z["allit"], z["heads"], z["picks"], z["vals"], z["x"], z["rows"]
    P, S = allit.shape
    base = sp.r - sp.T @ x
    B = np.tile(base[:, None], (1, S))
    B[rows, :] += (vals - sp.r[rows]).T
    lb = np.zeros(n + m); ub = np.full(n + m, np.inf)
    lb[n:][sense == 'G'] = -np.inf; ub[n:][sense == 'G'] = 0.0
    ub[n:][sense == 'E'] = 0.0
    F = {}
    def put(name, p, val):
        F.setdefault(name, np.zeros((P, S)))[p] = val
    for p in range(P):
        h = heads[p]
        Bm = np.zeros((m, m)); st = h >= n
        Bm[:, ~st] = W[:, h[~st]]
        Bm[h[st] - n, np.nonzero(st)[0]] = 1.0
        Binv = np.linalg.inv(Bm)
        xb = Binv @ B
        l = lb[h][:, None]; u = ub[h][:, None]
        v = np.maximum(np.maximum(l - xb, xb - u), 0.0); v[np.isnan(v)] = 0
        viol = v > 1e-9
        rn = np.sqrt((Binv ** 2).sum(1))[:, None]
        put("sum", p, (v * viol).sum(0)); put("cnt", p, viol.sum(0))
        put("sum_dse", p, (v / rn).sum(0)); put("sq_dse", p, ((v / rn) ** 2).sum(0))
        for t in taus: put(f"cnt>{t}", p, (v > t).sum(0))
        put("logsum", p, np.log1p(v).sum(0))
        put("sqrt", p, np.sqrt(v).sum(0))
    cols = np.arange(S)
    print(tag, "gpu picks", allit[picks, cols].mean(), "hindsight", allit.min(0).mean())
    def ev(key, name):
        pk = np.argmin(key, 0)
        print(f"{tag} {name:34s} {allit[pk, cols].mean():.2f}", flush=True)
    for k in F: ev(F[k] + 1e-12 * F["sum"], k)
    for cw in [3, 10]:
        ev(F["sum"] + cw * F["cnt"], f"sum+{cw}cnt")
    for cw in [0.1, 1, 10]:
        ev(F["sum_dse"] + cw * F["cnt"], f"sum_dse+{cw}cnt")
    for t in taus:
        ev(F[f"cnt>{t}"] + 0.1 * F["cnt"] + 1e-3 * F["sum"], f"cnt>{t}+0.1cnt")
    ev(F["logsum"] + 0.0 * F["cnt"], "logsum")
    for a in [0.5, 1, 2]:
        ev(F["logsum"] + a * F["cnt"], f"logsum+{a}cnt")
    np.savez(f"gpurun_out/hs_feat_{tag}.npz", **F)
