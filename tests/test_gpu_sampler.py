"""On-device scenario sampler (rand(rng, sto) smps_sto.jl:117-149) against
the C oracle (oracle/sampler.c, pinned by the Philox4x32-10 known answers): DISCRETE and
UNIFORM elements bit-exact, NORMAL within 1e-12 (device log/cos vs glibc)."""
import numpy as np
import pytest

from tests import instances as I

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["storm", "ssn", "transship", "lands"])
def test_device_sampler_matches_oracle(name):
    from oracle import cpu
    from sqlp_amd import twosd
    inst = I.load(name)
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    ctx.set_distributions(inst["sto"])
    epi = twosd.sdEpigraph(ctx, 1.0, 0.0)
    N, seed = 20000, 0x5EED1234ABCDEF
    twosd.add_sampled_scenarios(epi, N, seed, first_index=7)
    assert epi.num_scenarios == N and epi.total_scenario_weight == N
    got = twosd.get_scenarios(epi)
    ref = cpu.sample_deltas(inst["sto"], ctx.positions, ctx.template_values, N, seed, 7) + ctx.template_values
    kinds = np.array([inst["sto"].indep[p][0] for p in ctx.positions])
    exact = kinds != "NORMAL"
    np.testing.assert_array_equal(got[:, exact], ref[:, exact])
    if (~exact).any():
        np.testing.assert_allclose(got[:, ~exact], ref[:, ~exact], rtol=1e-12, atol=1e-12)


def test_device_sampler_sharding_and_solve():
    """Shards (first_index) reproduce one stream; sampled scenarios solve like host ones."""
    from sqlp_amd import twosd
    inst = I.load("storm")
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    ctx.set_distributions(inst["sto"])
    x = I.x_ev("storm")
    from sqlp_amd import smps
    ctx.compute_basis(x, smps.mean_values(inst["sto"]))
    a = twosd.sdEpigraph(ctx, 1.0, 0.0)
    b = twosd.sdEpigraph(ctx, 1.0, 0.0)
    twosd.add_sampled_scenarios(a, 4096, 99)
    twosd.add_sampled_scenarios(b, 1000, 99, first_index=0)
    twosd.add_sampled_scenarios(b, 3096, 99, first_index=1000)
    np.testing.assert_array_equal(twosd.get_scenarios(a), twosd.get_scenarios(b))
    obj_a, _, _, st = twosd.solve_batch(a, x, want_pi=False)
    obj_h, _, _, st_h = ctx.solve_values(x, twosd.get_scenarios(a), want_pi=False)
    assert (st == 0).all() and (st_h == 0).all()
    np.testing.assert_allclose(obj_a, obj_h, rtol=1e-12)


@pytest.mark.parametrize("name", ["lands", "storm"])
def test_evaluate_sampled(name):
    """evaluate(sp1, sp2, sto, x; N) on device-drawn scenarios == the same scenarios
    (oracle stream) solved through solve_values and summed in order (smps_routines.jl:79)."""
    from oracle import cpu
    from sqlp_amd import smps, twosd
    inst = I.load(name)
    ctx = twosd.SDContext(inst["sp2"], inst["sto"])
    ctx.set_distributions(inst["sto"])
    x = I.x_ev(name)
    ctx.compute_basis(x, smps.mean_values(inst["sto"]))
    c1 = np.ones(len(x))
    N, seed = 30000, 4242
    val = twosd.evaluate_sampled(ctx, c1, x, N, seed)
    vals = cpu.sample_deltas(inst["sto"], ctx.positions, ctx.template_values, N, seed) + ctx.template_values
    ref = twosd.evaluate(ctx, c1, x, vals)
    assert abs(val - ref) <= 1e-10 * (1 + abs(ref))
    # two shards of the stream add up to the whole
    h = N // 3
    s_a = twosd.evaluate_sampled(ctx, np.zeros(len(x)), x, N, seed, 0, h)
    s_b = twosd.evaluate_sampled(ctx, np.zeros(len(x)), x, N, seed, h, N - h)
    assert abs(float(np.dot(c1, x)) + s_a + s_b - val) <= 1e-10 * (1 + abs(val))
