"""CPU oracle for the TwoSD scenario-subproblem + cut-generation hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is product code: only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import, link or execute it, and only as the checker (or the timed CPU
baseline), never as the thing measured or shipped.

Contents (each module cites the reference file:line it restates; paths are
relative to the reference repo yhz0/SQLP @ 2025-02-19):

* ``smps_ref``   -- SMPS cor/tim/sto parsing + stage split
                    (src/smps/smps_cor.jl, smps_tim.jl, smps_sto.jl, smps_prob.jl)
* ``twosd_ref``  -- dual-vertex set, delta coefficients, eval_dual,
                    argmax_procedure, build_sasa_cut
                    (src/sd_algorithm/dual_set.jl, subprob.jl, epigraph.jl)
* ``lp_highs``   -- the second-stage LP of ``solve_problem!``
                    (src/smps/smps_routines.jl:50-62) solved by HiGHS (scipy 1.15.3),
                    duals mapped to JuMP's sign convention.
* ``cpu_lp.c``   -- plain-C warm-started dual simplex (product-form update from a
                    shared optimal basis) + argmax/cut loops in reference order;
                    the timed CPU baseline ("port") of bench.py.

Parity pinning: the reference is Julia 1.9.3 + JuMP/GLPK, which is not installed
here (no julia binary, no network) -- nothing was denied, the toolchain is absent.
The oracle is pinned by the reference's own known-answer tests (test/*.jl, lands)
and by HiGHS-generated golden vectors committed under tests/golden/.
"""
