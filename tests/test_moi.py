"""MOI adapter (socp_amd.moi, mirror of src/moi.jl): model packing on CPU, solves on the GPU.

The reference's MOI tests do not exist (test/runtests.jl builds Problems
directly), so the packing is checked against the runtests.jl problems written
in MOI form (moi.jl:142-160 sign convention: A, G = -F; b, h = f0) and the
solves against the reference's own x* (runtests.jl:142,165,185) and the oracle.
"""
import numpy as np
import pytest

import socp_amd as S
from socp_amd import moi as M
from problems import kat_problem


def model_from_dense(c, A, b, G, h, cones, sense=M.MIN_SENSE, shuffle=False, **opts):
    """Write (c, A, b, G, h, cones) as MOI constraints: b - A x ∈ Zeros, h_c - G_c x ∈ K_c."""
    o = M.Optimizer(**opts)
    n = len(c)
    v = o.add_variables(n)
    cc = -np.asarray(c) if sense == M.MAX_SENSE else np.asarray(c)
    o.set_objective_sense(sense)
    o.set_objective_function(M.saf([(v[j], cc[j]) for j in range(n) if cc[j] != 0], 0.0))
    cons = []
    if len(b):
        cons.append(("Z", M.Zeros(len(b)), -np.asarray(A), np.asarray(b)))
    for kind, offs, dim in cones:
        st = M.Nonnegatives(dim) if kind == S.CONE_POC else M.SecondOrderCone(dim)
        cons.append(("K", st, -np.asarray(G)[offs:offs + dim], np.asarray(h)[offs:offs + dim]))
    if shuffle:
        cons = cons[::-1]
    cis = []
    for _, st, F, f0 in cons:
        rows = [(i + 1, v[j], F[i, j]) for i in range(F.shape[0]) for j in range(n) if F[i, j] != 0]
        cis.append(o.add_constraint(M.vaf(rows, f0), st))
    return o, v, cis


@pytest.mark.parametrize("name", ["soc1", "soc2", "soc3"])
def test_pack_reference_problems(kats, name):
    cones, c, A, b, G, h = kat_problem(kats[name])
    o, _, _ = model_from_dense(c, A, b, G, h, cones)
    d = o.build()
    assert np.array_equal(d.c, c) and np.array_equal(d.G, G) and np.array_equal(d.h, h)
    assert np.array_equal(d.A, A.reshape(-1, len(c))) and np.array_equal(d.b, b)
    assert S._as_cone_list(d.cones) == [tuple(x) for x in cones]


def test_pack_order_duplicates_sense_and_no_poc():
    o = M.Optimizer()
    x, y, t = o.add_variables(3)
    # SOC added before the Nonnegatives rows: the rows still come after them (moi.jl:108)
    ci_q = o.add_constraint(M.vaf([(1, t, 1.0), (2, y, 1.0), (3, x, 0.5), (3, x, 0.5)], [0, 0, 0]),
                            M.SecondOrderCone(3))
    ci_l = o.add_constraint(M.vaf([(1, t, -1.0)], [5.0]), M.Nonnegatives(1))
    o.set_objective_sense(M.MAX_SENSE)
    o.set_objective_function(M.saf([(x, 1.0), (y, 1.0), (t, -1.0)], 2.5))
    d = o.build()
    assert ci_q.value == 0 and ci_l.value == 0 and o._constroffset(ci_q) == 1
    assert np.array_equal(d.G, [[0, 0, 1], [0, 0, -1], [0, -1, 0], [-1, 0, 0]])  # duplicates summed
    assert np.array_equal(d.h, [5, 0, 0, 0])
    assert np.array_equal(d.c, [-1, -1, 1])  # MAX_SENSE negates (moi.jl:199)
    assert S._as_cone_list(d.cones) == [(S.CONE_POC, 0, 1), (S.CONE_SOC, 1, 3)]
    o2 = M.Optimizer()
    a, b2 = o2.add_variables(2)
    o2.add_constraint(M.vaf([(1, a, 1.0), (2, b2, 1.0)], [0, 0]), M.SecondOrderCone(2))
    assert S._as_cone_list(o2.build().cones) == [(S.CONE_SOC, 0, 2)]  # no POC(0,0)


def test_rejects_unsupported_and_bad_input():
    o = M.Optimizer()
    x = o.add_variable()
    assert o.supports_constraint(M.VectorAffineFunction, M.SecondOrderCone)
    assert not o.supports_constraint(M.ScalarAffineFunction, M.Nonnegatives)
    with pytest.raises(ValueError):
        o.add_constraint(M.vaf([(2, x, 1.0)], [0.0]), M.Nonnegatives(1))
    with pytest.raises(ValueError):
        o.add_constraint(M.vaf([(1, M.VariableIndex(7), 1.0)], [0.0]), M.Nonnegatives(1))
    with pytest.raises(ValueError):
        o.build()  # no conic rows
    assert o.termination_status() == M.OPTIMIZE_NOT_CALLED
    o.empty_()
    assert o.is_empty()


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["soc1", "soc2", "soc3"])
def test_optimize_reference_problems(kats, oracle, name):
    q = kats[name]
    cones, c, A, b, G, h = kat_problem(q)
    o, v, cis = model_from_dense(c, A, b, G, h, cones, shuffle=True)
    o.optimize()
    assert o.termination_status() == "OPTIMAL" and o.result_count() == 1
    x = o.variable_primal(v)
    assert np.linalg.norm(x - np.array(q["x_expect"])) < q["tol"]  # runtests.jl's own assertion
    r = oracle.solve_trace(cones, c, A, b, G, h)
    assert o.barrier_iterations() == r["iters"]
    assert np.abs(x - r["x"]).max() <= 1e-3
    # same numbers as the Problem/solve_socp surface on the packed data (shuffle=True
    # adds the SOC constraints in reverse, so their rows are permuted vs the kat problem)
    d = o.data
    prob = S.Problem(d.c, d.A, d.b, d.G, d.h, S._as_cone_list(d.cones))
    st = S.solve_socp(prob, S.SolverState(prob, S.DenseSolver(prob)))
    assert np.array_equal(x, st.x)
    assert abs(o.objective_value() - c @ x) < 1e-12
    for ci in cis:  # constraint primal/dual are the rows of s/z (y for Zeros)
        rows = o._rows(ci)
        if ci.set_type is M.Zeros:
            assert np.array_equal(o.constraint_dual(ci), st.y[rows])
            assert not o.constraint_primal(ci).any()
        else:
            assert np.array_equal(o.constraint_primal(ci), st.s[rows])
            assert np.array_equal(o.constraint_dual(ci), st.z[rows])


@pytest.mark.gpu
def test_optimize_batched_matches_single(kats):
    """Perturbed copies of SOC3 (+ SOC1, another structure class) in one call:
    each model equals its own single optimize (batch independence)."""
    rng = np.random.default_rng(7)
    models = []
    for i in range(40):
        name = "soc3" if i % 4 else "soc1"
        cones, c, A, b, G, h = kat_problem(kats[name])
        c = c + 0.1 * rng.standard_normal(c.shape)
        h = h + 0.1 * np.abs(rng.standard_normal(h.shape))
        models.append((model_from_dense(c, A, b, G, h, cones)[:2], (cones, c, A, b, G, h)))
    M.optimize_batched([m[0][0] for m in models])
    for (o, v), data in models:
        xb, itb = o.variable_primal(v), o.barrier_iterations()
        o2, v2, _ = model_from_dense(*data[1:], data[0])
        o2.optimize()
        assert np.array_equal(xb, o2.variable_primal(v2)) and itb == o2.barrier_iterations()
        assert o.termination_status() == o2.termination_status()
