"""Pipelined host ingest (socp_ingest_*): host batches
through double-buffered pinned staging, the next batch's host-to-device copy
(and CSC packing) overlapping the current solve.

Gate: every batch's results are bitwise those of the synchronous
socp_batch_solve_ex on the same inputs -- dense form, zero-copy form (arrays
written straight into the pinned slot), CSC form (packed on the device), the
blocked kernel, partial batches -- and the misuse cases fail loudly.
"""
import numpy as np
import pytest

import socp_amd as S
from socp_amd.configs import C2

pytestmark = pytest.mark.gpu

KEYS = ("x", "y", "z", "s", "iters", "status", "res")


def host_batch(cfg, B, first):
    d = S.generate(cfg.cones, B, cfg.n, cfg.m, cfg.k, cfg.seed, first_problem=first)
    return [t.cpu().numpy() for t in d]


def sync_solve(cfg, data, sing, **kw):
    c, A, b, G, h = data
    return S.batch_solve(cfg.cones, cfg.n, cfg.m, cfg.k, c, A, b, G, h, sing, res=True, **kw)


def same(got, ref):
    for key in KEYS:
        assert np.array_equal(got[key], ref[key]), key


def test_pipelined_dense_batches_bitwise():
    cfg, B = C2, 2048
    ing = S.Ingest(cfg.cones, cfg.n, cfg.m, cfg.k, B)
    batches = [host_batch(cfg, B, i * B) for i in range(4)]
    sing = np.zeros(B, np.uint8)
    kw = dict(maxit=8, tol=0.0)
    # submit 0, 1 / wait 0, submit 2 / wait 1, submit 3 / wait 2, 3: two in flight
    t = [ing.submit(*batches[0], sing, **kw), ing.submit(*batches[1], sing, **kw)]
    outs = []
    for i in range(2, 4):
        outs.append(ing.wait(t[i - 2], res=True))
        t.append(ing.submit(*batches[i], sing, **kw))
    outs += [ing.wait(t[2], res=True), ing.wait(t[3], res=True)]
    for data, got in zip(batches, outs):
        same(got, sync_solve(cfg, data, sing, **kw))


def test_zero_copy_inputs_and_partial_batch():
    cfg, Bmax, B = C2, 1024, 700
    ing = S.Ingest(cfg.cones, cfg.n, cfg.m, cfg.k, Bmax)
    data = host_batch(cfg, B, 5000)
    slot = ing.next_inputs()
    for key, arr in zip(("c", "A", "b", "G", "h"), data):
        slot[key][:arr.size] = arr
    views = [slot[key][:arr.size] for key, arr in zip(("c", "A", "b", "G", "h"), data)]
    got = ing.wait(ing.submit(*views, None, maxit=6, tol=0.0), res=True)
    same(got, sync_solve(cfg, data, None, maxit=6, tol=0.0))  # sing = NULL: device cholesky(G'G) test
    assert ing.wait(ing.submit(*[v[:0] for v in views], None)) ["x"].size == 0  # empty batch


def test_csc_batches_bitwise():
    import scipy.sparse as sp
    cfg, B = C2, 512
    c, A, b, G, h = host_batch(cfg, B, 123)
    n, m, k = cfg.n, cfg.m, cfg.k
    rng = np.random.default_rng(0)
    # sparsify G (keep the structure the generator made feasible: drop 70% of
    # the off-diagonal entries of every problem's G) and keep A dense-as-CSC
    Gd = G.reshape(B, n, k).transpose(0, 2, 1).copy()  # per problem k x n
    mask = rng.random(Gd.shape) < 0.3
    Gd *= mask
    Gs = [sp.csc_matrix(Gd[p]) for p in range(B)]
    As = [sp.csc_matrix(A.reshape(B, n, m)[p].T) for p in range(B)]
    Gflat = np.concatenate([M.toarray().ravel(order="F") for M in Gs])
    Aflat = np.concatenate([M.toarray().ravel(order="F") for M in As])
    sing = np.zeros(B, np.uint8)
    ing = S.Ingest(cfg.cones, n, m, k, B)
    t0 = ing.submit_csc(c, b, h, None, As, Gs, maxit=5, tol=0.0)
    t1 = ing.submit_csc(c, b, h, sing, As, Gs, index_base=0, maxit=5, tol=0.0)
    r0, r1 = ing.wait(t0, res=True), ing.wait(t1, res=True)
    ref = sync_solve(cfg, (c, Aflat, b, Gflat, h), None, maxit=5, tol=0.0)
    same(r0, ref)
    ref1 = sync_solve(cfg, (c, Aflat, b, Gflat, h), sing, maxit=5, tol=0.0)
    same(r1, ref1)


def test_blocked_kernel_through_ingest():
    cfg, B = C2, 64
    data = host_batch(cfg, B, 77)
    ing = S.Ingest(cfg.cones, cfg.n, cfg.m, cfg.k, B, force_large=True)
    got = ing.wait(ing.submit(*data, None, maxit=4, tol=0.0), res=True)
    same(got, sync_solve(cfg, data, None, maxit=4, tol=0.0, force_large=True))


def test_misuse_fails_loudly():
    import scipy.sparse as sp
    cfg, B = C2, 16
    data = host_batch(cfg, B, 0)
    ing = S.Ingest(cfg.cones, cfg.n, cfg.m, cfg.k, B)
    t0 = ing.submit(*data)
    t1 = ing.submit(*data)
    with pytest.raises(S.SocpError, match="outstanding"):
        ing.submit(*data)
    ing.wait(t0)
    ing.wait(t1)
    with pytest.raises(S.SocpError, match="batch outside"):
        big = host_batch(cfg, 2 * B, 0)
        ing.submit(*big)
    # a CSC batch whose row index is out of range reports at wait
    c, A, b, G, h = data
    Gs = [sp.csc_matrix(G.reshape(B, cfg.n, cfg.k)[p].T) for p in range(B)]
    As = [sp.csc_matrix(A.reshape(B, cfg.n, cfg.m)[p].T) for p in range(B)]
    nz, colptr, rowval, nzval = S._csc_arrays(Gs, cfg.k, cfg.n, 1)
    rowval = rowval.copy()
    rowval[3] = cfg.k + 5
    t = ing.submit_csc(c, b, h, None, As, (nz, colptr, rowval, nzval))
    with pytest.raises(S.SocpError, match="row index"):
        ing.wait(t)
