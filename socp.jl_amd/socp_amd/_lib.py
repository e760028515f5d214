"""ctypes binding of libsocp.so (include/socp.h).

The HIP library is the only compute path: if it is missing or no GPU is
present, every solve raises.  There is no CPU fallback in the product.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))  # socp.jl_amd/
LIB_PATH = os.environ.get("SOCP_AMD_LIB") or os.path.join(_PKG_ROOT, "lib", "libsocp.so")
HEADER = os.path.join(os.path.dirname(_PKG_ROOT), "include", "socp.h")

# return codes / statuses / flags (include/socp.h)
SOCP_OK, SOCP_E_INVALID, SOCP_E_UNSUPPORTED, SOCP_E_HIP, SOCP_E_NOMEM = 0, -1, -2, -3, -4
CONVERGED, MAXIT, CHOL_H_FAILED, CHOL_S_FAILED, DOMAIN_ERROR = 0, 1, 2, 3, 4
CONE_POC, CONE_SOC = 0, 1
F_DEVICE_PTRS, F_WARM_START, F_FORCE_LARGE, F_EXPLICIT_INVERSE = 1, 2, 4, 8

EXPORTED = [
    "socp_last_error", "socp_version", "socp_params_default", "socp_ctx_create",
    "socp_ctx_destroy", "socp_ctx_sync", "socp_ctx_stream", "socp_ctx_set_stream", "socp_ctx_reset_stream", "socp_supported",
    "socp_batch_solve", "socp_batch_solve_ex", "socp_batch_kkt_solve", "socp_generate",
    "socp_last_kernel_ms", "socp_last_kernel_name", "socp_kernel_times", "socp_debug_set_kkt_dump",
    "socp_debug_set_stamps", "socp_pack_csc", "socp_comm_unique_id", "socp_comm_init",
    "socp_comm_destroy", "socp_allgather_status", "socp_allgather_outcomes",
    "socp_dense_create", "socp_dense_setup_iter", "socp_dense_solve_kkt", "socp_dense_h2d_bytes",
    "socp_dense_record_bytes", "socp_dense_destroy",
    "socp_ingest_create", "socp_ingest_next_inputs", "socp_ingest_submit", "socp_ingest_submit_csc",
    "socp_ingest_wait", "socp_ingest_destroy",
    "socp_sqr_supported", "socp_sqr_create", "socp_sqr_setup_iter", "socp_sqr_solve_kkt", "socp_sqr_factor",
    "socp_sqr_scaling", "socp_sqr_h2d_bytes", "socp_sqr_record_bytes", "socp_sqr_destroy",
    "socp_sqr_solve_socp",
]

OUTCOME_BYTES = 32  # sizeof(socp_outcome): int32 status, int32 iters, double rd, rp, gap
MAX_BATCH = 2**31 - 1  # device problem indices are int32


class SocpError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libsocp error {code}: {msg}")
        self.code = code


class Dims(C.Structure):
    _fields_ = [("batch", C.c_int64), ("n", C.c_int32), ("m", C.c_int32), ("k", C.c_int32),
                ("ncones", C.c_int32)]


class Params(C.Structure):
    _fields_ = [("maxit", C.c_int32), ("sigma_exp", C.c_int32), ("tol", C.c_double),
                ("step", C.c_double), ("init_eps", C.c_double), ("flags", C.c_int32),
                ("reserved", C.c_int32)]


def default_params(**kw) -> Params:
    """socp_params with the reference constants (solver.jl:105,122,133,146,91)."""
    p = Params(40, 3, 1e-5, 0.99, 1e-10, 0, 0)
    for key, v in kw.items():
        setattr(p, key, v)
    return p


_lib = None


def load():
    """Load libsocp.so; raises (loudly) if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libsocp.so not built ({LIB_PATH}); run __graft_entry__.build()")
    # One HIP runtime per process: torch ships its own libamdhip64 (same soname
    # as /opt/rocm's).  Loading torch first makes libsocp bind to that copy, so
    # device pointers, streams and contexts are shared; loading libsocp first
    # would bring up a second runtime and torch would then see no GPU.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    vp, i32p, dp, u8p = C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p
    L.socp_last_error.restype = C.c_char_p
    L.socp_version.restype = C.c_char_p
    L.socp_params_default.argtypes = [C.POINTER(Params)]
    L.socp_ctx_create.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
    L.socp_ctx_destroy.argtypes = [vp]
    L.socp_ctx_sync.argtypes = [vp]
    L.socp_ctx_stream.argtypes = [vp]
    L.socp_ctx_stream.restype = C.c_void_p
    L.socp_ctx_set_stream.argtypes = [vp, vp]
    L.socp_ctx_reset_stream.argtypes = [vp]
    L.socp_supported.argtypes = [C.POINTER(Dims)]
    common = [vp, C.POINTER(Dims), i32p, i32p, i32p]
    L.socp_batch_solve.argtypes = common + [dp] * 5 + [u8p, C.POINTER(Params)] + [dp] * 4 + [i32p, i32p]
    L.socp_batch_solve_ex.argtypes = common + [dp] * 5 + [u8p, C.POINTER(Params)] + [dp] * 4 + [i32p, i32p, dp]
    L.socp_batch_kkt_solve.argtypes = common + [dp, dp, u8p] + [dp] * 2 + [dp] * 4 + [dp] * 4 + [i32p, C.c_int32]
    L.socp_generate.argtypes = common + [C.c_uint64, C.c_int64] + [dp] * 5
    L.socp_last_kernel_ms.argtypes = [vp, C.POINTER(C.c_float)]
    L.socp_kernel_times.argtypes = [vp, C.POINTER(C.c_float), C.c_int]
    L.socp_last_kernel_name.argtypes = [vp]
    L.socp_last_kernel_name.restype = C.c_char_p
    L.socp_debug_set_kkt_dump.argtypes = [vp]
    L.socp_debug_set_stamps.argtypes = [vp]
    L.socp_pack_csc.argtypes = [vp, C.c_int64, C.c_int32, C.c_int32, vp, vp, vp, vp, C.c_int32, vp]
    if hasattr(L, "socp_dense_create"):  # split plugin entries (absent from older A/B builds)
        L.socp_dense_create.argtypes = common + [dp, dp, u8p, C.c_int32, C.POINTER(C.c_void_p)]
        L.socp_dense_setup_iter.argtypes = [vp, dp, dp, i32p]
        L.socp_dense_solve_kkt.argtypes = [vp] + [dp] * 8 + [i32p]
        L.socp_dense_h2d_bytes.argtypes = [vp, C.POINTER(C.c_int64)]
        L.socp_dense_record_bytes.argtypes = [vp]
        L.socp_dense_record_bytes.restype = C.c_int64
        L.socp_dense_destroy.argtypes = [vp]
    if hasattr(L, "socp_sqr_create"):  # rank-update plugin (absent from older A/B builds)
        L.socp_sqr_supported.argtypes = [C.POINTER(Dims)]
        L.socp_sqr_create.argtypes = common + [dp, dp, u8p, C.c_int32, C.POINTER(C.c_void_p)]
        L.socp_sqr_setup_iter.argtypes = [vp, dp, dp, i32p]
        L.socp_sqr_solve_kkt.argtypes = [vp] + [dp] * 8 + [i32p]
        L.socp_sqr_factor.argtypes = [vp, C.c_int64, dp]
        L.socp_sqr_scaling.argtypes = [vp, dp, dp, dp]
        L.socp_sqr_h2d_bytes.argtypes = [vp, C.POINTER(C.c_int64)]
        L.socp_sqr_record_bytes.argtypes = [vp]
        L.socp_sqr_record_bytes.restype = C.c_int64
        L.socp_sqr_destroy.argtypes = [vp]
        if hasattr(L, "socp_sqr_solve_socp"):
            L.socp_sqr_solve_socp.argtypes = [vp] + [dp] * 3 + [C.POINTER(Params)] + [dp] * 4 + [i32p, i32p, dp]
    if hasattr(L, "socp_ingest_create"):  # pipelined ingest (absent from older A/B builds)
        L.socp_ingest_create.argtypes = common + [C.c_int32, C.POINTER(C.c_void_p)]
        L.socp_ingest_next_inputs.argtypes = [vp] + [C.POINTER(C.c_void_p)] * 6
        L.socp_ingest_submit.argtypes = [vp, C.c_int64] + [dp] * 5 + [u8p, C.POINTER(Params), C.POINTER(C.c_int64)]
        L.socp_ingest_submit_csc.argtypes = ([vp, C.c_int64] + [dp] * 3 + [u8p] + [vp] * 4 + [vp] * 4
                                             + [C.c_int32, C.POINTER(Params), C.POINTER(C.c_int64)])
        L.socp_ingest_wait.argtypes = [vp, C.c_int64] + [dp] * 4 + [i32p, i32p, dp]
        L.socp_ingest_destroy.argtypes = [vp]
    if hasattr(L, "socp_comm_init"):  # RCCL gather (absent from libraries built before it)
        L.socp_comm_unique_id.argtypes = [vp]
        L.socp_comm_init.argtypes = [vp, C.c_int, C.c_int, vp, C.POINTER(C.c_void_p)]
        L.socp_comm_destroy.argtypes = [vp]
        L.socp_allgather_status.argtypes = [vp, C.c_int64, vp, vp, vp]
        L.socp_allgather_outcomes.argtypes = [vp, C.c_int64, vp, vp, vp, vp]
    _lib = L
    return L


def check(rc: int):
    if rc != 0:
        raise SocpError(rc, load().socp_last_error().decode())


def ptr(a) -> C.c_void_p:
    """Raw pointer of a numpy array or a torch tensor (host or device); None passes NULL."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return C.c_void_p(a.ctypes.data)
    return C.c_void_p(a.data_ptr())  # torch.Tensor


class Context:
    """One socp_ctx (a HIP stream on one device); one per host thread."""

    def __init__(self, device: int = 0):
        L = load()
        h = C.c_void_p()
        check(L.socp_ctx_create(device, C.byref(h)))
        self.handle = h
        self.device = device

    def close(self):
        if self.handle:
            load().socp_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def sync(self):
        check(load().socp_ctx_sync(self.handle))

    @property
    def stream(self) -> int:
        return load().socp_ctx_stream(self.handle)

    def set_stream(self, stream) -> None:
        """Issue the context's work on `stream` (a hipStream_t as int; 0 is the
        null stream, torch's default) -- socp_ctx_set_stream."""
        check(load().socp_ctx_set_stream(self.handle, C.c_void_p(stream) if stream else None))

    def reset_stream(self) -> None:
        """Back to the context's own stream (socp_ctx_reset_stream)."""
        check(load().socp_ctx_reset_stream(self.handle))

    def bind_torch_stream(self) -> None:
        """Order the context's work on torch's current stream of its device, so
        tensors torch produced just before a call are complete when the solver
        reads them, and torch work issued after it sees the results."""
        import torch
        self.set_stream(torch.cuda.current_stream(self.device).cuda_stream)

    def last_kernel_ms(self) -> float:
        v = C.c_float()
        check(load().socp_last_kernel_ms(self.handle, C.byref(v)))
        return float(v.value)

    def kernel_times(self, n: int) -> list:
        """Main-kernel times (ms) of the last min(n, 64) timed launches, oldest
        first (socp_kernel_times): no host synchronisation between launches."""
        buf = (C.c_float * max(n, 1))()
        got = load().socp_kernel_times(self.handle, buf, n)
        check(min(got, 0))
        return [float(buf[i]) for i in range(got)]

    def last_kernel_name(self) -> str:
        return load().socp_last_kernel_name(self.handle).decode()


_default_ctx = {}


def default_context(device: int = 0) -> Context:
    if device not in _default_ctx:
        _default_ctx[device] = Context(device)
    return _default_ctx[device]
