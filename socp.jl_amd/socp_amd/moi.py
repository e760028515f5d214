"""MathOptInterface-style adapter for the HIP dense path.

Mirror of the reference's `Socp.Optimizer` (`src/moi.jl`), whose data model is
ECOS's: every constraint is `f(x) = Fx + f0 ∈ K`, stored as `b - A x ∈ Zeros`
(rows of A, b) or `h - G x ∈ K` (rows of G, h) with `A, G = -F` and
`b, h = f0` (`moi.jl:142-160`).  Nonnegatives rows come first, then the
second-order cones in the order they were added (`moi.jl:101-116`), so the cone
tuple is `POC(0, l), SOC(l, q1), SOC(l+q1, q2), ...` (`moi.jl:212-217`).

Differences from the reference, each fixing a defect that keeps `moi.jl` from
running:

* `optimize!` builds `SolverState(prob, DenseSolver(prob))` and runs on the
  GPU (the reference calls `solve_socp(prob, SparseSolver(prob))`, a solver
  object where a `SolverState` is expected, `moi.jl:220`).
* No `POC(0, 0)` when the model has no Nonnegatives rows (`moi.jl:212`).
* `scalecoef` (undefined in the reference, `moi.jl:251,257`) is the identity:
  it only rescales PSD cones, which this solver does not support.
* The dual of a `Zeros` constraint is `y` (the reference reads `z`,
  `moi.jl:254`); termination/objective getters exist.

Beyond the reference: `optimize_batched(optimizers)` solves many models in
one device launch per structure class (same n, equality rows, Nonnegatives
length and SOC dimensions) — the batched dense path this framework exists for.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass, field

import numpy as np

from . import CONVERGED, MAXIT, CHOL_H_FAILED, CHOL_S_FAILED, DOMAIN_ERROR, POC, SOC, batch_solve

MIN_SENSE, MAX_SENSE, FEASIBILITY_SENSE = "MIN_SENSE", "MAX_SENSE", "FEASIBILITY_SENSE"
OPTIMIZE_NOT_CALLED = "OPTIMIZE_NOT_CALLED"
TERMINATION = {CONVERGED: "OPTIMAL", MAXIT: "ITERATION_LIMIT", CHOL_H_FAILED: "NUMERICAL_ERROR",
               CHOL_S_FAILED: "NUMERICAL_ERROR", DOMAIN_ERROR: "NUMERICAL_ERROR"}


# ------------------------------------------------------------------ MOI types
@dataclass(frozen=True)
class VariableIndex:
    value: int  # 1-based, as MOI.VariableIndex


@dataclass(frozen=True)
class ScalarAffineTerm:
    coefficient: float
    variable: VariableIndex


@dataclass(frozen=True)
class VectorAffineTerm:
    output_index: int  # 1-based row of the vector function
    scalar_term: ScalarAffineTerm


@dataclass
class ScalarAffineFunction:
    terms: list
    constant: float = 0.0


@dataclass
class VectorAffineFunction:
    terms: list
    constants: list


@dataclass(frozen=True)
class Zeros:
    dimension: int


@dataclass(frozen=True)
class Nonnegatives:
    dimension: int


@dataclass(frozen=True)
class SecondOrderCone:
    dimension: int


@dataclass(frozen=True)
class ConstraintIndex:
    set_type: type
    value: int  # the reference's ci.value: offset inside the set's row class (moi.jl:101-116)


@dataclass
class _Con:
    f: VectorAffineFunction
    s: object
    ci: ConstraintIndex


@dataclass
class _Solution:
    x: np.ndarray
    y: np.ndarray
    z: np.ndarray
    s: np.ndarray
    iters: int
    status: int


@dataclass
class ModelData:
    """The packed problem of one model (moi.jl:24-37, dense here)."""
    c: np.ndarray
    A: np.ndarray  # f x n, row-major
    b: np.ndarray
    G: np.ndarray  # (l + q) x n, row-major
    h: np.ndarray
    cones: tuple
    objconstant: float = 0.0
    signature: tuple = field(default=())


class Optimizer:
    """`Socp.Optimizer` (moi.jl:57-66) over the GPU dense path.  Keyword options:
    `maxit` (default 40, solver.jl:105), `tol` (1e-5, solver.jl:122), `ctx`."""

    def __init__(self, **options):
        self.options = dict(options)
        self.empty_()

    # -- MOI.SolverName / supports / is_empty / empty! (moi.jl:68-91)
    solver_name = "SOCP.jl (MI355X dense path)"

    @staticmethod
    def supports_constraint(ftype, stype) -> bool:
        return ftype is VectorAffineFunction and stype in (Zeros, Nonnegatives, SecondOrderCone)

    def is_empty(self) -> bool:
        return self.nvars == 0 and not self.cons and self.sense != MAX_SENSE and self.sol is None

    def empty_(self):
        self.nvars = 0
        self.cons: list[_Con] = []
        self.f = self.l = self.q = 0
        self.qa: list[int] = []
        self.sense = MIN_SENSE
        self.objective = ScalarAffineFunction([], 0.0)
        self.sol: _Solution | None = None
        self.data: ModelData | None = None

    # -- variables / objective
    def add_variable(self) -> VariableIndex:
        self.nvars += 1
        return VariableIndex(self.nvars)

    def add_variables(self, n: int) -> list:
        return [self.add_variable() for _ in range(n)]

    def set_objective_sense(self, sense):
        self.sense = sense  # MOIU.allocate(::ObjectiveSense) (moi.jl:187-189)

    def set_objective_function(self, f: ScalarAffineFunction):
        self.objective = f

    # -- constraints: _allocate_constraint (moi.jl:96-116)
    def add_constraint(self, f: VectorAffineFunction, s) -> ConstraintIndex:
        if not self.supports_constraint(type(f), type(s)):
            raise TypeError(f"unsupported constraint {type(f).__name__} in {type(s).__name__}")
        if len(f.constants) != s.dimension:
            raise ValueError("function output dimension does not match the set dimension")
        for t in f.terms:
            if not (1 <= t.output_index <= s.dimension):
                raise ValueError(f"output index {t.output_index} outside 1:{s.dimension}")
            if not (1 <= t.scalar_term.variable.value <= self.nvars):
                raise ValueError(f"unknown variable {t.scalar_term.variable.value}")
        if isinstance(s, Zeros):
            ci = ConstraintIndex(Zeros, self.f)
            self.f += s.dimension
        elif isinstance(s, Nonnegatives):
            ci = ConstraintIndex(Nonnegatives, self.l)
            self.l += s.dimension
        else:
            if s.dimension < 1:
                raise ValueError("SecondOrderCone needs dimension >= 1")
            self.qa.append(s.dimension)
            ci = ConstraintIndex(SecondOrderCone, self.q)
            self.q += s.dimension
        self.cons.append(_Con(f, s, ci))
        self.sol = None
        return ci

    def _constroffset(self, ci: ConstraintIndex) -> int:
        # constroffset (moi.jl:96,102,108): SOC rows follow all Nonnegatives rows
        return self.l + ci.value if ci.set_type is SecondOrderCone else ci.value

    # -- copy_to / load (moi.jl:142-200): the packed dense problem
    def build(self) -> ModelData:
        n, f, k = self.nvars, self.f, self.l + self.q
        if n == 0:
            raise ValueError("model has no variables")
        if k == 0:
            raise ValueError("the dense path needs at least one conic (Nonnegatives or SOC) row")
        A, b = np.zeros((f, n)), np.zeros(f)
        G, h = np.zeros((k, n)), np.zeros(k)
        for con in self.cons:
            off = self._constroffset(con.ci)
            M, v = (A, b) if con.ci.set_type is Zeros else (G, h)
            rows = off + np.arange(con.s.dimension)
            v[rows] = np.asarray(con.f.constants, dtype=np.float64)
            if con.f.terms:
                I = np.array([off + t.output_index - 1 for t in con.f.terms])
                J = np.array([t.scalar_term.variable.value - 1 for t in con.f.terms])
                V = np.array([-t.scalar_term.coefficient for t in con.f.terms], dtype=np.float64)
                np.add.at(M, (I, J), V)  # MOIU.canonical merges duplicate terms (moi.jl:143)
        c0 = np.zeros(n)
        for t in self.objective.terms:
            c0[t.variable.value - 1] += t.coefficient
        c = -c0 if self.sense == MAX_SENSE else c0  # moi.jl:199
        cones = ((POC(0, self.l),) if self.l else ()) + tuple(
            SOC(self.l + sum(self.qa[:i]), d) for i, d in enumerate(self.qa))
        sig = (n, f, self.l, tuple(self.qa))
        self.data = ModelData(c, A, b, G, h, cones, float(self.objective.constant), sig)
        return self.data

    # -- optimize! (moi.jl:203-222)
    def optimize(self):
        optimize_batched([self])

    def _set_solution(self, x, y, z, s, iters, status):
        self.sol = _Solution(np.array(x), np.array(y), np.array(z), np.array(s), int(iters), int(status))

    # -- getters (moi.jl:240-272)
    def _need_sol(self):
        if self.sol is None:
            raise RuntimeError("optimize() has not been called since the model last changed")
        return self.sol

    def termination_status(self) -> str:
        return TERMINATION[self.sol.status] if self.sol is not None else OPTIMIZE_NOT_CALLED

    def result_count(self) -> int:
        return 1 if self.sol is not None else 0  # moi.jl:272 (always 1 there)

    def barrier_iterations(self) -> int:
        return self._need_sol().iters

    def variable_primal(self, vi):
        sol = self._need_sol()
        if isinstance(vi, (list, tuple)):
            return np.array([sol.x[v.value - 1] for v in vi])
        return float(sol.x[vi.value - 1])

    def objective_value(self) -> float:
        sol = self._need_sol()
        c0 = -self.data.c if self.sense == MAX_SENSE else self.data.c
        return float(c0 @ sol.x + self.data.objconstant)

    def _rows(self, ci: ConstraintIndex):
        for con in self.cons:
            if con.ci == ci:
                off = self._constroffset(ci)
                return off + np.arange(con.s.dimension)
        raise KeyError(ci)

    def constraint_primal(self, ci: ConstraintIndex) -> np.ndarray:
        sol, rows = self._need_sol(), self._rows(ci)
        if ci.set_type is Zeros:  # moi.jl:245-248
            return np.zeros(len(rows))
        return sol.s[rows].copy()  # moi.jl:253-257, scalecoef = identity

    def constraint_dual(self, ci: ConstraintIndex) -> np.ndarray:
        sol, rows = self._need_sol(), self._rows(ci)
        return (sol.y if ci.set_type is Zeros else sol.z)[rows].copy()


def optimize_batched(optimizers, ctx=None):
    """`MOI.optimize!` for many models at once: models are grouped by structure
    (n, equality rows, Nonnegatives length, SOC dimensions) and each group is one
    `socp_batch_solve` launch.  Per-model options `maxit`/`tol` must agree within a group."""
    groups: "OrderedDict[tuple, list]" = OrderedDict()
    for o in optimizers:
        d = o.build()
        key = d.signature + (int(o.options.get("maxit", 40)), float(o.options.get("tol", 1e-5)))
        groups.setdefault(key, []).append(o)
    for key, opts in groups.items():
        n, f, l, qa = key[:4]
        maxit, tol = key[4], key[5]
        k = l + sum(qa)
        ds = [o.data for o in opts]
        sing = np.array([_sing(d.G) for d in ds], np.uint8)
        c = np.concatenate([d.c for d in ds])
        A = np.concatenate([d.A.ravel(order="F") for d in ds]) if f else None
        b = np.concatenate([d.b for d in ds]) if f else None
        G = np.concatenate([d.G.ravel(order="F") for d in ds])
        h = np.concatenate([d.h for d in ds])
        out = batch_solve(ds[0].cones, n, f, k, c, A, b, G, h, sing, maxit=maxit, tol=tol,
                          ctx=ctx if ctx is not None else opts[0].options.get("ctx"))
        for i, o in enumerate(opts):
            o._set_solution(out["x"][i * n:(i + 1) * n], out["y"][i * f:(i + 1) * f],
                            out["z"][i * k:(i + 1) * k], out["s"][i * k:(i + 1) * k],
                            out["iters"][i], out["status"][i])


def _sing(G) -> bool:
    """`sing` of Problem (Socp.jl:49-56): cholesky(G'G) throws."""
    try:
        np.linalg.cholesky(G.T @ G)
        return False
    except np.linalg.LinAlgError:
        return True


def vaf(rows, constants):
    """Shorthand: VectorAffineFunction from [(output_index, VariableIndex, coef), ...]."""
    return VectorAffineFunction([VectorAffineTerm(i, ScalarAffineTerm(float(a), v)) for i, v, a in rows],
                                [float(x) for x in constants])


def saf(terms, constant=0.0):
    """Shorthand: ScalarAffineFunction from [(VariableIndex, coef), ...]."""
    return ScalarAffineFunction([ScalarAffineTerm(float(a), v) for v, a in terms], float(constant))
