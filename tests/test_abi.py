"""The C-ABI library (libsocp.so) and the host-side mirror, without a GPU."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import socp_amd as S
from socp_amd import _lib
from socp_amd.configs import CONFIGS
from problems import kat_problem


def _header_functions():
    txt = open(_lib.HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(socp_[a-z0-9_]+)\s*\(", txt)))


def test_library_built_and_loads():
    assert os.path.exists(_lib.LIB_PATH), "run __graft_entry__.build() first"
    L = _lib.load()
    assert L.socp_version().decode().startswith("socp-mi355x")


def test_exports_every_declared_symbol():
    L = C.CDLL(_lib.LIB_PATH)
    declared = _header_functions()
    assert len(declared) >= 14
    missing = [f for f in declared if not hasattr(L, f)]
    assert not missing, missing
    assert set(_lib.EXPORTED) == set(declared)


def test_default_params_are_reference_constants():
    p = _lib.Params()
    _lib.load().socp_params_default(C.byref(p))
    # solver.jl:105 (maxit 40), :122 (tol 1e-5), :133 (sigma^3), :146 (0.99), :91,97 (1e-10)
    assert (p.maxit, p.sigma_exp, p.tol, p.step, p.init_eps, p.flags) == (40, 3, 1e-5, 0.99, 1e-10, 0)


def test_supported_dims():
    L = _lib.load()
    for name, ok in (("C0b", True), ("C1", True), ("C2", True), ("C4", True)):
        cfg = CONFIGS[name]
        d = _lib.Dims(cfg.batch, cfg.n, cfg.m, cfg.k, len(cfg.cones))
        assert bool(L.socp_supported(C.byref(d))) == ok, name
    # beyond the blocked kernel: n or m > 2048, or more than 64 cones
    for n, m, k, nc in ((2049, 0, 2050, 1), (64, 2100, 128, 1), (256, 0, 130, 65)):
        assert not L.socp_supported(C.byref(_lib.Dims(1, n, m, k, nc))), (n, m, k)
    # n, m > 512: the blocked kernel's windowed wide panels (Cholesky order)
    for n, m, k, nc in ((600, 0, 601, 1), (2048, 512, 2100, 8), (64, 600, 128, 1), (2048, 2048, 2100, 8)):
        assert L.socp_supported(C.byref(_lib.Dims(1, n, m, k, nc))), (n, m, k)
    # k-vectors over the 160 KiB LDS run with the vectors in HBM (the GV kernels)
    for n, m, k, nc in ((512, 64, 1000, 8), (64, 16, 4096, 4), (64, 16, 1 << 21, 4)):
        assert L.socp_supported(C.byref(_lib.Dims(1, n, m, k, nc))), (n, m, k)
    # beyond the blocked kernel's 32-bit LDS / vector offsets (LARGE_KMAX)
    for n, m, k, nc in ((64, 16, (1 << 21) + 1, 4), (512, 64, 1 << 30, 8), (8, 0, 2**31 - 1, 1)):
        assert not L.socp_supported(C.byref(_lib.Dims(1, n, m, k, nc))), (n, m, k)


def test_null_context_is_an_api_error():
    L = _lib.load()
    d = _lib.Dims(1, 3, 0, 4, 2)
    rc = L.socp_batch_solve(None, C.byref(d), None, None, None, None, None, None, None, None, None, None,
                            None, None, None, None, None, None)
    assert rc == _lib.SOCP_E_INVALID
    assert b"ctx" in L.socp_last_error()


def test_problem_mirror_asserts_and_sing(kats):
    # Problem(c, A, b, G, h, cones): shape asserts (Socp.jl:43-47) and `sing` (Socp.jl:49-56)
    cones, c, A, b, G, h = kat_problem(kats["soc3"])
    p = S.Problem(c, A, b, G, h, cones)
    assert (p.n, p.m, p.k, p.sing) == (3, 1, 7, False)
    with pytest.raises(AssertionError):
        S.Problem(c, A, b[:0], G, h, cones)
    with pytest.raises(AssertionError):
        S.Problem(c, A, b, G, h[:-1], cones)
    sing_prob = S.Problem(np.zeros(10), np.ones((8, 10)), np.ones(8), np.ones((3, 10)), np.ones(3), [S.SOC(0, 3)])
    assert sing_prob.sing
    with pytest.raises(AssertionError):
        S.State(p, np.zeros(2), np.zeros(1), np.zeros(7), np.zeros(7))


def test_cone_arrays():
    kind, offs, dim = S.cone_arrays([S.POC(0, 32), S.SOC(32, 32), (1, 64, 32)])
    assert kind.tolist() == [0, 1, 1] and offs.tolist() == [0, 32, 64] and dim.tolist() == [32, 32, 32]


def test_flop_and_byte_model():
    import bench
    # C1 134.3 K, C2 939.3 K, C4 344.8 M flop; C2 63.1 KB
    assert abs(bench.flops_per_problem_iter(32, 8, 48) - 134.3e3) < 0.1e3
    assert abs(bench.flops_per_problem_iter(64, 16, 96) - 939.3e3) < 0.1e3
    assert abs(bench.flops_per_problem_iter(512, 64, 640) - 344.8e6) < 0.1e6
    assert abs(bench.bytes_per_problem_iter(64, 16, 96) - 63.1e3) < 0.1e3


def test_host_arrays_are_size_checked():
    """every array is checked against (B, n, m, k) before the C ABI
    reads it (a short host array would be an out-of-bounds read)."""
    from socp_amd.configs import C1
    cfg = C1
    B, n, m, k = 3, cfg.n, cfg.m, cfg.k
    good = dict(c=np.zeros(B * n), A=np.zeros(B * m * n), b=np.zeros(B * m), G=np.zeros(B * k * n),
                h=np.zeros(B * k))
    for key, short in (("A", B * m * n - 1), ("b", B * m + 1), ("G", B * k * n - n), ("h", B * k - 1)):
        arrs = dict(good)
        arrs[key] = np.zeros(short)
        with pytest.raises(ValueError, match=key):
            S.batch_solve(cfg.cones, n, m, k, arrs["c"], arrs["A"], arrs["b"], arrs["G"], arrs["h"])
    with pytest.raises(ValueError, match="sing"):
        S.batch_solve(cfg.cones, n, m, k, *good.values(), sing=np.zeros(B + 1, np.uint8))
    with pytest.raises(ValueError, match="multiple"):
        S.batch_solve(cfg.cones, n, m, k, np.zeros(B * n + 1), *list(good.values())[1:])
    with pytest.raises(ValueError, match="warm_z"):
        S.batch_solve(cfg.cones, n, m, k, *good.values(),
                      warm=(np.zeros(B * n), np.zeros(B * m), np.zeros(B * k - 2), np.zeros(B * k)))
    with pytest.raises(ValueError, match="dz"):
        S.batch_kkt_solve(cfg.cones, n, m, k, good["A"], good["G"], None, np.zeros(B * k), np.zeros(B * k),
                          np.zeros(B * n), np.zeros(B * m), np.zeros(B * k + 3), np.zeros(B * k))


def test_sqr_supported_dims():
    # the rank-update plugin: n, m <= 1024, k <= 4096, the vectors' LDS layout
    # <= 160 KiB (socp_sqr.hpp; factors beyond the LDS live in the record)
    L = _lib.load()
    for name in ("C0b", "C1", "C2", "C4"):  # C4 (n = 512): the factors in the record
        cfg = CONFIGS[name]
        d = _lib.Dims(cfg.batch, cfg.n, cfg.m, cfg.k, len(cfg.cones))
        assert L.socp_sqr_supported(C.byref(d)), name
    assert L.socp_sqr_supported(C.byref(_lib.Dims(1, 65, 0, 10, 1)))
    assert L.socp_sqr_supported(C.byref(_lib.Dims(1, 150, 102, 50, 1)))  # runtests.jl:204-244
    assert L.socp_sqr_supported(C.byref(_lib.Dims(1, 160, 160, 256, 16)))
    for n, m, k in ((161, 0, 10), (64, 161, 10), (64, 0, 257), (400, 100, 500), (1024, 1024, 1100)):
        assert L.socp_sqr_supported(C.byref(_lib.Dims(1, n, m, k, 1))), (n, m, k)
    for n, m, k in ((1025, 0, 1100), (64, 1025, 10), (64, 0, 4097), (1024, 1024, 4096)):
        assert not L.socp_sqr_supported(C.byref(_lib.Dims(1, n, m, k, 1))), (n, m, k)
