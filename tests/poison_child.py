"""Child process of tests/test_gpu_poison.py (run as `python -m tests.poison_child OUT.npz`).

The allocation-poison hook (TWOSD_POISON / TWOSD_POISON_FAMILY, api.hip) is read once when the
library first allocates, so the parent sets it in this process's environment before anything
loads the library.  The workload is the refresh path of the bench on storm: two pool refreshes
(the second composes from device-built start bases), the two-level candidate lists after each,
a keyed solve + push of 4,096 scenarios and a cut with its argmax.  Everything a kernel reads
must have been written by a kernel first, so every output must be bit-identical with and
without the fill."""
import sys

import numpy as np


def main(out_path):
    from sqlp_amd import smps, twosd
    from tests import instances as I
    from tests.test_gpu_pool_refresh import _sd_x

    inst = I.load("storm")
    x_ev = I.x_ev("storm")
    x2 = _sd_x(3)
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    ctx.compute_basis(x_ev, smps.mean_values(inst["sto"]))
    ctx.set_distributions(inst["sto"])
    tr = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(tr, 4096, seed=31)
    ev = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(ev, 4096, seed=32)
    res = {"x2": x2}
    for tag, xx in (("a", x_ev), ("b", x2)):
        P = ctx.pool_refresh(tr, xx, 0, 4096, 512)
        ctx.pool_build_candidates(tr, xx, 0, 4096, 128, 160)
        res[f"heads_{tag}"] = np.stack([ctx.pool_get(p) for p in range(P)])
    V = twosd.sdDualVertexSet(ctx)
    obj, st, _ = twosd.solve_push(ev, x2, 0, 4096)
    res["obj"], res["status"] = obj, st
    res["iters"], _ = ctx.last_lp_iters(4096)
    res["picks"] = ctx.last_pool_picks(4096)
    res["V"] = V.matrix()
    cut, mv, ma = twosd._build_cut(ev, x2, 0.0, want_argmax=True)
    res.update(alpha=np.array([cut.alpha]), beta=cut.beta, max_val=mv, max_arg=ma)
    np.savez(out_path, **res)


if __name__ == "__main__":
    main(sys.argv[1])
