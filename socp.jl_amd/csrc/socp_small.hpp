// socp_small.hpp — the register-resident batched dense SOCP IPM kernel (gfx950).
//
// One 64-lane wavefront owns one problem for its whole solve (persistent
// one-wave blocks pull problem indices from an atomic work counter).  The
// problem's G (k x n, the dominant data: 48 KiB at n=64,k=96) is loaded from
// HBM once per solve and stays in AGPRs for every iteration, laid out as the
// B-operand fragment of v_mfma_f64_16x16x4_f64:
//     lane (g = lane>>4, cl = lane&15) holds G[4p+g][16q+cl] in G[p][q].
// Per iteration (reference solver.jl:105-151):
//   - NT scaling (scalings.jl:22-110) with per-cone segmented DPP scans;
//   - residuals (solver.jl:110-122) from register G;
//   - H = X'X with X = W^-1 G generated in registers and contracted by f64
//     MFMA: the reference's iWiW GEMM, G'*iWiW and *G (scalings.jl:108,
//     densesolver.jl:42-43) done structurally; +A'A if sing (:44-46);
//   - the explicit inverse Li = H^-1 (densesolver.jl:47-48) by an in-register
//     symmetric Gauss-Jordan sweep whose pivots are the Cholesky pivots, so
//     positive-definiteness fails exactly where cholesky! would;
//   - ALi' = Li A' and S = A Li A' on MFMA, S^-1 by the same sweep (:49-51);
//   - two KKT solves (densesolver.jl:54-90) and the step/update.
// LDS (<40 KiB per wave at n=64) holds only vectors, A and broadcast scratch,
// so four one-wave blocks (one per SIMD) share a CU.
//
// Code-size discipline: the driver is a micro-phase loop in which the cone
// vector op, the factorisation, the KKT solve body and the residuals each
// have exactly one inlined instance (no calls: a call would force the live
// H/Li tiles out of registers), keeping the instruction stream cache-resident.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace socp {

typedef double d4 __attribute__((ext_vector_type(4)));

constexpr int MAXC = 64;   // cone table size in the kernel arguments
constexpr int NCS = 8;     // cones supported by the register-resident kernel
constexpr int KMAX = 128;  // k supported by the register-resident kernel
constexpr int POC_K = 0, SOC_K = 1;

struct ConeTable {
  int32_t nc;
  int32_t kind[MAXC];
  int32_t offs[MAXC];
  int32_t dim[MAXC];
};

enum { MODE_SOLVE = 0, MODE_KKT = 1 };
enum { ST_CONVERGED = 0, ST_MAXIT = 1, ST_CHOL_H = 2, ST_CHOL_S = 3, ST_DOMAIN = 4 };
enum { F_WARM = 2 };

struct SmallArgs {
  int64_t B;
  int32_t n, m, k, nc;
  int32_t maxit, sigma_exp;
  double tol, step, init_eps;
  int32_t flags, mode, deg, pad0;
  const double *c, *A, *b, *G, *h;
  const uint8_t* sing;
  double *x, *y, *z, *s;
  int32_t *iters, *status;
  double* res;
  const double *dx, *dy, *dz, *ds;
  double *cx, *cy, *cz, *cs;
  int32_t* counter;
  double* dbg;                 // optional (KKT mode): per problem H[n*n], Li[n*n], lam[k], wb[k]
  unsigned long long* stamps;  // SOCP_DIAG builds: per-phase cycle totals
  ConeTable cones;
};

// ------------------------------------------------------------ LDS layout
// Fixed region (independent of the template shape):
enum : int {
  O_RC = 0,                  // rcode[KMAX]: cone*4 + type (0 POC, 1 SOC head, 2 SOC tail, 3 pad)
  O_COFF = O_RC + KMAX,      // cone offs[NCS]
  O_CDIM = O_COFF + NCS,     // cone dim[NCS]
  O_CKIND = O_CDIM + NCS,    // cone kind[NCS]
  O_MU = O_CKIND + NCS,      // mu per cone
  O_I1 = O_MU + NCS,         // 1/(1+wb0) per cone
  O_TOT = O_I1 + NCS,        // reduced values per cone [NCS][4]
  O_PART = O_TOT + 4 * NCS,  // per-slot partials [2][NCS][4]
  O_CST = O_PART + 8 * NCS,  // step-length scratch per cone [NCS][4]
  O_KV = O_CST + 4 * NCS,    // 16 k-vectors of KMAX
  O_FIXED_END = O_KV + 16 * KMAX
};
// k-vector ids
enum : int { KV_H, KV_Z, KV_S, KV_DZ, KV_DS, KV_RZ, KV_RS, KV_LAM, KV_WB, KV_CA, KV_CB, KV_K0,
             KV_K1, KV_K2, KV_T1, KV_T2 };
__host__ __device__ constexpr int kv(int id) { return O_KV + id * KMAX; }

template <int NQ, int NP, int MQ>
struct Shape {
  static constexpr int NPAD = 16 * NQ, KP = 4 * NP, MPAD = 16 * MQ, LDA = NPAD + 1;
  // sweep gather buffer: pivot column of the diagonal tile [16] + pivot row of
  // every tile of the panel slab [16 per tile]
  static constexpr int CB = 16 + (NPAD > MPAD ? NPAD : MPAD);
  static constexpr int O_A = O_FIXED_END;
  static constexpr int O_NV = O_A + MPAD * LDA;    // n-vectors: c x rd rx n0 tn
  static constexpr int O_MV = O_NV + 6 * NPAD;     // m-vectors: b y rp ry m0 tm
  static constexpr int O_U = O_MV + 6 * MPAD;      // U[NCS][NPAD]
  static constexpr int O_COL = O_U + NCS * NPAD;   // sweep column buffers [2][CB]
  static constexpr int O_TB = O_COL + 2 * CB;      // tile transpose [16][17]
  static constexpr int TOTAL = O_TB + 16 * 17;
  static constexpr int nv(int id) { return O_NV + id * NPAD; }
  static constexpr int mv(int id) { return O_MV + id * MPAD; }
};
enum : int { NV_C, NV_X, NV_RD, NV_RX, NV_N0, NV_TN };
enum : int { MV_B, MV_Y, MV_RP, MV_RY, MV_M0, MV_TM };

inline size_t small_lds_bytes(int NQ, int NP, int MQ) {
  int NPAD = 16 * NQ, MPAD = 16 * MQ, LDA = NPAD + 1, CB = 16 + (NPAD > MPAD ? NPAD : MPAD);
  int total = O_FIXED_END + MPAD * LDA + 6 * NPAD + 6 * MPAD + NCS * NPAD + 2 * CB + 16 * 17;
  return (size_t)total * sizeof(double);
}

// Diagnostic phase timing (separate build, -DSOCP_DIAG): per-phase s_memtime
// deltas accumulated per problem and added to a global table by lane 0.
#ifdef SOCP_DIAG
#define NSTAMP 12
#define STAMP_DECL uint64_t st_last = 0; uint64_t st_acc[NSTAMP] = {0};
#define STAMP_START_S(obj) do { __builtin_amdgcn_s_waitcnt(0); (obj).st_last = __builtin_amdgcn_s_memtime(); } while (0)
#define STAMP(i) do { __builtin_amdgcn_s_waitcnt(0); const uint64_t t_ = __builtin_amdgcn_s_memtime(); st_acc[i] += t_ - st_last; st_last = t_; } while (0)
#else
#define STAMP_DECL
#define STAMP_START_S(obj) do {} while (0)
#define STAMP(i) do {} while (0)
#endif
enum { SP_LOAD, SP_SCALING, SP_RESID, SP_U, SP_SYRK, SP_SWEEP_H, SP_SCHUR, SP_SOLVE, SP_STEP, SP_VOP,
       SP_STORE, SP_OTHER };

extern __shared__ double socp_lds[];
#define LDS(i) socp_lds[(i)]
#define SYNC() __syncthreads()

// A double pinned in two AGPRs (gfx950: VALU cannot read AGPRs; MFMA can).
// G lives here for the whole solve and is copied to VGPRs at each use.
struct AD {
  uint32_t lo, hi;
};
__device__ __forceinline__ void a_put(AD& r, double v) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(r.lo) : "v"((uint32_t)u));
  asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(r.hi) : "v"((uint32_t)(u >> 32)));
}
__device__ __forceinline__ double a_get(const AD& r) {
  uint32_t lo, hi;
  asm("v_accvgpr_read_b32 %0, %1" : "=v"(lo) : "a"(r.lo));
  asm("v_accvgpr_read_b32 %0, %1" : "=v"(hi) : "a"(r.hi));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// a_get for a value consumed directly as an MFMA A/B operand: v_accvgpr_read is
// a VALU write, and VALU write -> MFMA operand read needs 2 wait states, which
// hipcc does not insert for a producer inside inline asm (it pads one state).
__device__ __forceinline__ double a_get_mfma(const AD& r) {
  uint32_t lo, hi;
  asm("v_accvgpr_read_b32 %0, %2\n\tv_accvgpr_read_b32 %1, %3\n\ts_nop 1"
      : "=v"(lo), "=v"(hi)
      : "a"(r.lo), "a"(r.hi));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Scheduling fence: keeps the scheduler from hoisting the next unrolled step's
// loads above this point (with H pinned in VGPRs and G in AGPRs, hoisting
// across steps is what overflows the register file).
#define SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ constexpr int tri(int i, int j) { return i * (i + 1) / 2 + j; }
__device__ __forceinline__ double sel4(d4 t, int r) {
  double v = t[0];
  v = (r == 1) ? t[1] : v;
  v = (r == 2) ? t[2] : v;
  v = (r == 3) ? t[3] : v;
  return v;
}

// DPP move of a double (two 32-bit halves).  CTRL: 0x111+s = row_shr:s+1,
// 0x142 = row_bcast:15, 0x143 = row_bcast:31 (GFX9 DPP); RM = row mask.
template <int CTRL, int RM>
__device__ __forceinline__ double dpp(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int l2 = __builtin_amdgcn_update_dpp(0, lo, CTRL, RM, 0xF, false);
  const int h2 = __builtin_amdgcn_update_dpp(0, hi, CTRL, RM, 0xF, false);
  return __hiloint2double(h2, l2);
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// Lane ids re-read inside each phase (LANE_IDS shadows the members): values
// derived from them (4*pp + g, 16*ti + cl, ...) are then recomputed where they
// are used instead of being hoisted out of the persistent loop and kept live.
__device__ __forceinline__ int lane_fresh() {
  int v = (int)threadIdx.x;
  asm volatile("" : "+v"(v));
  return v;
}
#define LANE_IDS()                      \
  const int lane = lane_fresh();        \
  const int g = lane >> 4, cl = lane & 15; \
  (void)g; (void)cl

// Wave-uniform copies.  LLVM's divergence analysis treats every LDS or global
// load as divergent; a branch on such a value (the sweep's pivot test, the
// per-problem `sing` flag, the phase number) is then compiled as exec-masked
// straight-line code: every arm runs and the live ranges of all arms merge.
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ double uni(double v) {
  const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
  const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
  return __hiloint2double(hi, lo);
}

// Inclusive segmented scan over the 64 lanes with DPP (row_shr 1,2,4,8 then
// row_bcast 15/31): lane l accumulates lanes [max(ssl, 0) .. l] with op
// (sum, or max when mx).  ssl = first lane of l's segment.
template <int V>
__device__ __forceinline__ void dpp_scan(double (&x)[V], int lane, int ssl, bool mx) {
  const int rl = lane & 15;
#define SOCP_SCAN_STEP(CTRL, RM, OK)                                 \
  {                                                                  \
    const bool ok_ = (OK);                                           \
    _Pragma("unroll") for (int v = 0; v < V; ++v) {                  \
      const double y = dpp<CTRL, RM>(x[v]);                          \
      const double r = mx ? fmax(x[v], y) : x[v] + y;                \
      x[v] = ok_ ? r : x[v];                                         \
    }                                                                \
  }
  SOCP_SCAN_STEP(0x111, 0xF, rl >= 1 && lane - 1 >= ssl)
  SOCP_SCAN_STEP(0x112, 0xF, rl >= 2 && lane - 2 >= ssl)
  SOCP_SCAN_STEP(0x114, 0xF, rl >= 4 && lane - 4 >= ssl)
  SOCP_SCAN_STEP(0x118, 0xF, rl >= 8 && lane - 8 >= ssl)
  SOCP_SCAN_STEP(0x142, 0xA, ((lane >> 4) & 1) && ((lane & ~15) - 1 >= ssl))
  SOCP_SCAN_STEP(0x143, 0xC, lane >= 32 && 31 >= ssl)
#undef SOCP_SCAN_STEP
}

// whole-wave sum / max (scan to lane 63, broadcast through an SGPR)
__device__ __forceinline__ double wsum(double v) {
  double x[1] = {v};
  dpp_scan<1>(x, threadIdx.x, 0, false);
  return readlane_d(x[0], 63);
}
__device__ __forceinline__ double wmax(double v) {
  double x[1] = {v};
  dpp_scan<1>(x, threadIdx.x, 0, true);
  return readlane_d(x[0], 63);
}

// x^e for an integer exponent (Julia's ^(::Float64, ::Integer); e = 3 is x*x*x)
__device__ __forceinline__ double ipow(double x, int e) {
  if (e == 3) return x * x * x;
  double r = 1.0, b = x;
  for (int q = e; q > 0; q >>= 1) {
    if (q & 1) r *= b;
    b *= b;
  }
  return r;
}

// pivot reciprocal: v_rcp_f64 + two Newton steps (within 1 ulp of 1/d)
__device__ __forceinline__ double recip(double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  e = fma(-d, r, 1.0);
  return fma(r, e, r);
}

// Reduce-scatter over the 16 lanes of a row (xor masks 8,4,2,1): on return the
// lane holds in P[0..CF) the full row-sums of entries base+j.
template <int C, int M>
__device__ __forceinline__ void rs16(double* P, int cl, int& base) {
  if constexpr (M == 0) {
    return;
  } else if constexpr (C % 2 == 0) {
    constexpr int H = C / 2;
    const bool hi = (cl & M) != 0;
#pragma unroll
    for (int j = 0; j < H; ++j) {
      double mine = hi ? P[H + j] : P[j];
      double other = hi ? P[j] : P[H + j];
      P[j] = mine + __shfl_xor(other, M);
    }
    if (hi) base += H;
    rs16<H, M / 2>(P, cl, base);
  } else {
#pragma unroll
    for (int j = 0; j < C; ++j) P[j] += __shfl_xor(P[j], M);
    rs16<C, M / 2>(P, cl, base);
  }
}
template <int C, int M>
struct RSCount {
  static constexpr int value =
      (M == 0) ? C : ((C % 2 == 0) ? RSCount<C / 2, M / 2>::value : RSCount<C, M / 2>::value);
};
template <int C>
struct RSCount<C, 0> {
  static constexpr int value = C;
};

// cone vector operations (one instance, Small::vop)
enum : int { VOP_SCALE, VOP_ISCALE, VOP_PAIR, VOP_IPROD, VOP_VPROD, VOP_SCALING, VOP_STEP1,
             VOP_STEP2, VOP_MAXSTEP };

struct VopResult {
  double r0, r1;
  int dom;
};

// driver micro-phases
enum : int {
  MP_SINGTEST, MP_SINGTEST_POST, MP_FACTOR, MP_INIT, MP_INIT_RHS, MP_INIT_POST, MP_INIT_SHIFT,
  MP_ITER, MP_ITER_B, MP_ITER_C, MP_KKT, MP_KKT_B, MP_KKT_POST,
  MP_S0, MP_S1, MP_S2, MP_S3, MP_S4, MP_S5, MP_S6, MP_S7,
  MP_POST_A, MP_POST_B, MP_POST_C, MP_POST_D, MP_AFF_E
};

template <int NQ, int NP, int MQ>
struct Small {
  using SH = Shape<NQ, NP, MQ>;
  static constexpr int NT = NQ * (NQ + 1) / 2;
  static constexpr int MT = MQ * (MQ + 1) / 2;
  static constexpr int NPAD = SH::NPAD, KP = SH::KP, MPAD = SH::MPAD, LDA = SH::LDA;
  static constexpr int O_A = SH::O_A, O_U = SH::O_U, O_COL = SH::O_COL, O_TB = SH::O_TB;
  static constexpr int C_ = SH::nv(NV_C), X_ = SH::nv(NV_X), RD = SH::nv(NV_RD),
                       RX = SH::nv(NV_RX), N0 = SH::nv(NV_N0), TN = SH::nv(NV_TN);
  static constexpr int B_ = SH::mv(MV_B), Y_ = SH::mv(MV_Y), RP = SH::mv(MV_RP),
                       RY = SH::mv(MV_RY), M0 = SH::mv(MV_M0);
  static constexpr int H_ = kv(KV_H), Z_ = kv(KV_Z), S_ = kv(KV_S), DZ = kv(KV_DZ),
                       DS = kv(KV_DS), RZ = kv(KV_RZ), RS = kv(KV_RS), LAM = kv(KV_LAM),
                       WB = kv(KV_WB), CA = kv(KV_CA), CBV = kv(KV_CB), K0 = kv(KV_K0),
                       K1 = kv(KV_K1), K2 = kv(KV_K2), T1 = kv(KV_T1), T2 = kv(KV_T2);

  const SmallArgs& a;
  const int lane, g, cl;
  const int n, m, k, nc;
  bool sing;
  int64_t dbg_p = 0;
  // compact-layout element info (element i = 64*s + lane): cone, type code
  // (0 POC, 1 SOC head, 2 SOC tail, 3 none), cone offset, scan segment
  // start / last lane within the slot
  int ci[2], kd[2], eo[2], ssl[2], sle[2];
  STAMP_DECL

  AD G[NP][NQ];  // AGPR-resident
  d4 T[NT];
  d4 Sv[MT];

  __device__ __forceinline__ Small(const SmallArgs& args)
      : a(args), lane(threadIdx.x), g(threadIdx.x >> 4), cl(threadIdx.x & 15),
        n(args.n), m(args.m), k(args.k), nc(args.nc) {}

  // ---------------------------------------------------------------- setup
  __device__ __forceinline__ void init_tables() {
    if (lane < nc) {
      LDS(O_COFF + lane) = a.cones.offs[lane];
      LDS(O_CDIM + lane) = a.cones.dim[lane];
      LDS(O_CKIND + lane) = a.cones.kind[lane];
    }
    for (int i = lane; i < KMAX; i += 64) {
      int code = 3;
      if (i < k) {
        for (int c = 0; c < nc; ++c) {
          const int o = a.cones.offs[c], d = a.cones.dim[c];
          if (i >= o && i < o + d) {
            code = c * 4 + (a.cones.kind[c] == POC_K ? 0 : (i == o ? 1 : 2));
            break;
          }
        }
      }
      LDS(O_RC + i) = (double)code;
    }
    SYNC();
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = 64 * s + lane;
      const bool ev = i < k;
      const int code = ev ? (int)LDS(O_RC + i) : 3;
      const int c = ev ? (code >> 2) : 0;
      ci[s] = c;
      kd[s] = ev ? (code & 3) : 3;
      const int o = ev ? (int)LDS(O_COFF + c) : i;
      const int d = ev ? (int)LDS(O_CDIM + c) : 1;
      eo[s] = o;
      const int st = o > 64 * s ? o : 64 * s;
      const int en = (o + d) < 64 * (s + 1) ? (o + d) : 64 * (s + 1);
      ssl[s] = ev ? st - 64 * s : lane;
      sle[s] = ev ? en - 1 - 64 * s : -1;
    }
  }

  __device__ __forceinline__ void load_problem(int64_t p) {
    LANE_IDS();
    const double* Gp = a.G + p * (int64_t)k * n;
    // padding (row >= k or col >= n) reads element 0 and is zeroed with an
    // integer mask: no per-element exec mask is materialised
#pragma unroll
    for (int pp = 0; pp < NP; ++pp) {
      const int row = 4 * pp + g;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int col = 16 * q + cl;
        const int ok = (row < k) & (col < n);
        const int64_t idx = ok ? (int64_t)col * k + row : 0;
        const uint64_t bits = (uint64_t)__double_as_longlong(Gp[idx]) & (0ull - (uint64_t)ok);
        a_put(G[pp][q], __longlong_as_double((long long)bits));
      }
    }
    for (int e = lane; e < 16 * KMAX; e += 64) LDS(O_KV + e) = 0.0;
    for (int e = lane; e < SH::O_COL - O_A; e += 64) LDS(O_A + e) = 0.0;
    SYNC();
    const double* Ap = a.A + p * (int64_t)m * n;
    for (int e = lane; e < m * n; e += 64) {
      const int i = e % m, j = e / m;
      LDS(O_A + i * LDA + j) = Ap[e];
    }
    for (int j = lane; j < n; j += 64) LDS(C_ + j) = a.c[p * n + j];
    for (int i = lane; i < m; i += 64) LDS(B_ + i) = a.b[p * m + i];
    for (int i = lane; i < k; i += 64) LDS(H_ + i) = a.h[p * k + i];
    SYNC();
  }

  __device__ __forceinline__ double e_of(int i) const {
    const int code = (int)LDS(O_RC + i) & 3;
    return (code == 0 || code == 1) ? 1.0 : 0.0;
  }

  // W = I: the initial-point system (solver.jl:68-84) is the KKT system with
  // W = I, lam = e, ds = 0.
  __device__ __forceinline__ void scaling_identity() {
    for (int i = lane; i < k; i += 64) {
      const double e = e_of(i);
      LDS(WB + i) = e;
      LDS(LAM + i) = e;
      LDS(CA + i) = 1.0;
      LDS(CBV + i) = 0.0;
    }
    if (lane < nc) {
      LDS(O_MU + lane) = 1.0;
      LDS(O_I1 + lane) = 0.5;
    }
    for (int e = lane; e < NCS * NPAD; e += 64) LDS(O_U + e) = 0.0;
    SYNC();
  }

  // ------------------------------------------------------ cone vector ops
  // scale!/iscale! (scalings.jl:112-173), iprod!/vprod! (vectors.jl:58-125),
  // compute_scaling (scalings.jl:22-99), compute_step/scmax (mats.jl:30-86,
  // in two rounds STEP1/STEP2), max_step (mats.jl:1-28).  a, b, o1, o2 are
  // LDS offsets of k-vectors.  Exactly one instance (called from run()).
  __device__ __forceinline__ VopResult vop(int op, int a_, int b_, int o1, int o2) {
    LANE_IDS();
    double v[2][3];
    bool mxp = false;
    int nvals = 1;
    VopResult R = {0.0, 0.0, 0};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = 64 * s + lane;
      const bool tail = kd[s] == 2, hd = kd[s] == 1, poc = kd[s] == 0;
      double v0 = 0.0, v1 = 0.0, v2 = 0.0;
      if (op == VOP_SCALE || op == VOP_ISCALE) {
        if (tail) v0 = LDS(WB + i) * LDS(a_ + i);
      } else if (op == VOP_PAIR) {
        if (tail) {
          v0 = LDS(WB + i) * LDS(a_ + i);
          v1 = LDS(WB + i) * LDS(b_ + i);
        }
      } else if (op == VOP_IPROD) {
        const double li = LDS(LAM + i);
        if (tail) {
          v0 = li * li;
          v1 = LDS(a_ + i) * li;
        }
      } else if (op == VOP_VPROD) {
        if (tail || hd) v0 = LDS(a_ + i) * LDS(b_ + i);
      } else if (op == VOP_SCALING) {  // a = z, b = s
        if (tail) {
          const double zi = LDS(a_ + i), si = LDS(b_ + i);
          v0 = zi * zi;
          v1 = si * si;
          v2 = zi * si;
        }
      } else if (op == VOP_STEP1) {  // scmax(l, a), scmax(l, b): first round
        const double li = LDS(LAM + i);
        if (tail) {
          v0 = li * li;
          v1 = li * LDS(a_ + i);
          v2 = li * LDS(b_ + i);
        } else if (poc) {
          v0 = -LDS(a_ + i) / li;
          v1 = -LDS(b_ + i) / li;
        }
      } else if (op == VOP_STEP2) {  // second round: r2s of both directions
        if (tail) {
          const int o = eo[s], c = ci[s];
          const double av = LDS(O_CST + c * 4), ra = LDS(O_CST + c * 4 + 1),
                       rb = LDS(O_CST + c * 4 + 2);
          const double l0 = LDS(LAM + o), li = LDS(LAM + i);
          const double csa = (ra + LDS(a_ + o)) / (av * l0 + 1.0);
          const double csb = (rb + LDS(b_ + o)) / (av * l0 + 1.0);
          const double qa = av * (LDS(a_ + i) - csa * av * li);
          const double qb = av * (LDS(b_ + i) - csb * av * li);
          v0 = qa * qa;
          v1 = qb * qb;
        }
      } else if (op == VOP_MAXSTEP) {  // max_step(-a), max_step(a)
        const double xi = LDS(a_ + i);
        if (tail) v0 = xi * xi;
        if (poc) {
          v0 = xi;
          v1 = -xi;
        }
      }
      v[s][0] = v0;
      v[s][1] = v1;
      v[s][2] = v2;
    }
    if (op == VOP_PAIR || op == VOP_IPROD || op == VOP_STEP2 || op == VOP_MAXSTEP) nvals = 2;
    if (op == VOP_SCALING || op == VOP_STEP1) nvals = 3;
    mxp = (op == VOP_STEP1 || op == VOP_MAXSTEP);
    // ---- per-cone segmented reduction (DPP scan per slot, then per-cone totals)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (64 * s < k) {
        const bool mx = mxp && kd[s] == 0;
        if (nvals == 1) {
          double x[1] = {v[s][0]};
          dpp_scan<1>(x, lane, ssl[s], mx);
          v[s][0] = x[0];
        } else if (nvals == 2) {
          double x[2] = {v[s][0], v[s][1]};
          dpp_scan<2>(x, lane, ssl[s], mx);
          v[s][0] = x[0];
          v[s][1] = x[1];
        } else {
          dpp_scan<3>(v[s], lane, ssl[s], mx);
        }
        if (lane == sle[s]) {
#pragma unroll
          for (int q = 0; q < 3; ++q) LDS(O_PART + (s * NCS + ci[s]) * 4 + q) = v[s][q];
        }
      }
    }
    SYNC();
    if (lane < nc) {
      const int c = lane;
      const int o = (int)LDS(O_COFF + c), d = (int)LDS(O_CDIM + c);
      const bool mx = mxp && (int)LDS(O_CKIND + c) == POC_K;
      const int s0 = o >> 6, s1 = (o + d - 1) >> 6;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        double t = LDS(O_PART + (s0 * NCS + c) * 4 + q);
        if (s1 > s0) {
          const double u = LDS(O_PART + (s1 * NCS + c) * 4 + q);
          t = mx ? fmax(t, u) : t + u;
        }
        LDS(O_TOT + c * 4 + q) = t;
      }
    }
    SYNC();
    // ---- outputs
    bool dm = false;
    double best = -INFINITY, bp = -INFINITY;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (kd[s] == 3) continue;
      const int i = 64 * s + lane, c = ci[s], o = eo[s];
      const bool hd = kd[s] == 1, poc = kd[s] == 0;
      const double t0 = LDS(O_TOT + c * 4), t1 = LDS(O_TOT + c * 4 + 1), t2 = LDS(O_TOT + c * 4 + 2);
      if (op == VOP_SCALE || op == VOP_ISCALE || op == VOP_PAIR) {
        const double wi = LDS(WB + i), xi = LDS(a_ + i);
        double r;
        if (poc) {
          r = (op == VOP_ISCALE) ? (1.0 / wi) * xi : wi * xi;
        } else {
          const double mu = LDS(O_MU + c), wb0 = LDS(WB + o), x0 = LDS(a_ + o);
          if (op != VOP_ISCALE) {
            const double cst = x0 + t0 / (1.0 + wb0);
            r = hd ? mu * (wb0 * x0 + t0) : mu * (xi + cst * wi);
          } else {
            const double cst = -x0 + t0 / (1.0 + wb0);
            const double im = 1.0 / mu;
            r = hd ? im * (wb0 * x0 - t0) : im * (xi + cst * wi);
          }
        }
        if (op == VOP_PAIR) {
          const double x2 = LDS(b_ + i);
          double r2;
          if (poc) {
            r2 = (1.0 / wi) * x2;
          } else {
            const double mu = LDS(O_MU + c), wb0 = LDS(WB + o), x0 = LDS(b_ + o);
            const double cst = -x0 + t1 / (1.0 + wb0);
            const double im = 1.0 / mu;
            r2 = hd ? im * (wb0 * x0 - t1) : im * (x2 + cst * wi);
          }
          LDS(o2 + i) = r2;
        }
        LDS(o1 + i) = r;
      } else if (op == VOP_IPROD) {
        const double vi = LDS(a_ + i), li = LDS(LAM + i);
        double r;
        if (poc) {
          r = vi / li;
        } else {
          const double l0 = LDS(LAM + o), v0 = LDS(a_ + o);
          const double aa = l0 * l0 - t0;
          r = hd ? v0 * l0 / aa - t1 / aa : -(v0 * li / aa) + vi / l0 + li * t1 / (l0 * aa);
        }
        LDS(o1 + i) = r;
      } else if (op == VOP_VPROD) {
        const double ui = LDS(a_ + i), vi = LDS(b_ + i);
        double r;
        if (poc)
          r = ui * vi;
        else
          r = hd ? t0 : LDS(a_ + o) * vi + LDS(b_ + o) * ui;
        LDS(o1 + i) = r;
      } else if (op == VOP_SCALING) {
        // compute_scaling (scalings.jl:22-99) -> lam, wb, mu, 1/(1+wb0), and the
        // X = W^-1 G row coefficients: X[i,:] = ca[i] G[i,:] + cb[i] U[cone(i),:]
        const double zi = LDS(a_ + i), si = LDS(b_ + i);
        double wbi, li, cai, cbi;
        if (poc) {
          const double r = si / zi, pr = si * zi, ir = zi / si;
          dm |= (r < 0.0) || (pr < 0.0) || (ir < 0.0);
          wbi = sqrt(r);
          li = sqrt(pr);
          cai = sqrt(ir);
          cbi = 0.0;
        } else {
          const double z0 = LDS(a_ + o), s0 = LDS(b_ + o);
          const double onrmz = z0 * z0 - t0, onrms = s0 * s0 - t1;
          dm |= (onrmz < 0.0) || (onrms < 0.0);
          const double nrmz = sqrt(onrmz), nrms = sqrt(onrms);
          const double fz = 1.0 / nrmz, fs = 1.0 / nrms;
          const double zb0 = z0 * fz, sb0 = s0 * fs;
          const double nsum = zb0 * sb0 + t2 * fz * fs;
          const double garg = (1.0 + nsum) / 2.0;
          dm |= garg < 0.0;
          const double gamma = sqrt(garg);
          const double fg = 1.0 / (2.0 * gamma);
          const double wb0 = (sb0 + zb0) * fg;
          const double zbi = zi * fz, sbi = si * fs;
          wbi = hd ? wb0 : (sbi - zbi) * fg;
          const double ratio = nrms / nrmz, prod = nrms * nrmz;
          dm |= (ratio < 0.0) || (prod < 0.0);
          const double mu = sqrt(ratio);
          const double tmv1 = sqrt(prod);
          const double mult = tmv1 / (zb0 + sb0 + 2.0 * gamma);
          li = hd ? gamma * tmv1 : (sbi * (gamma + zb0) + zbi * (gamma + sb0)) * mult;
          const double im = 1.0 / mu;
          cai = hd ? -im : im;
          cbi = hd ? -(1.0 + wb0) * im : wbi * im;
          if (hd) {
            LDS(O_MU + c) = mu;
            LDS(O_I1 + c) = 1.0 / (1.0 + wb0);
          }
        }
        LDS(WB + i) = wbi;
        LDS(LAM + i) = li;
        LDS(CA + i) = cai;
        LDS(CBV + i) = cbi;
      } else if (op == VOP_STEP1) {
        if (hd) {
          const double l0 = LDS(LAM + o);
          const double ai = l0 * l0 - t0;
          dm |= ai < 0.0;
          const double av = 1.0 / sqrt(ai);
          LDS(O_CST + c * 4) = av;
          LDS(O_CST + c * 4 + 1) = av * l0 * LDS(a_ + o) - av * t1;
          LDS(O_CST + c * 4 + 2) = av * l0 * LDS(b_ + o) - av * t2;
        } else if (poc && i == o) {
          LDS(O_CST + c * 4 + 3) = fmax(t0, t1);
        }
      } else if (op == VOP_STEP2) {
        if (hd) {
          const double av = LDS(O_CST + c * 4);
          const double va = sqrt(t0) - av * LDS(O_CST + c * 4 + 1);
          const double vb = sqrt(t1) - av * LDS(O_CST + c * 4 + 2);
          best = fmax(best, fmax(va, vb));
        } else if (poc && i == o) {
          best = fmax(best, LDS(O_CST + c * 4 + 3));
        }
      } else if (op == VOP_MAXSTEP) {
        if (poc && i == o) {
          best = fmax(best, t0);
          bp = fmax(bp, t1);
        } else if (hd) {
          const double nr = sqrt(t0), x0 = LDS(a_ + o);
          best = fmax(best, nr + x0);
          bp = fmax(bp, nr - x0);
        }
      }
    }
    SYNC();
    R.dom = __any(dm) ? 1 : 0;
    if (op == VOP_STEP2) {
      double t = wmax(best);
      if (isnan(t)) t = -INFINITY;
      t = fmax(t, 0.0);
      R.r0 = (t == 0.0) ? 1.0 : fmin(1.0, 1.0 / t);
    } else if (op == VOP_MAXSTEP) {
      R.r0 = wmax(best);
      R.r1 = wmax(bp);
    }
    return R;
  }

  // U[c,:] = (sum_{i in cone c} w_i G[i,:]) / (1+wb0), w_head = -(1+wb0), w_tail = wb_i
  __device__ __forceinline__ void compute_U() {
    LANE_IDS();
    for (int c = 0; c < nc; ++c) {
      if (uni((int)LDS(O_CKIND + c)) != SOC_K) continue;
      const int o = uni((int)LDS(O_COFF + c)), d = uni((int)LDS(O_CDIM + c));
      const double wb0 = LDS(WB + o);
      double acc[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) acc[q] = 0.0;
#pragma unroll
      for (int pp = 0; pp < NP; ++pp) {
        if (4 * pp + 3 >= o && 4 * pp < o + d) {
          const int row = 4 * pp + g;
          const bool in = row >= o && row < o + d;
          const double w = in ? (row == o ? -(1.0 + wb0) : LDS(WB + row)) : 0.0;
#pragma unroll
          for (int q = 0; q < NQ; ++q) acc[q] = fma(w, a_get(G[pp][q]), acc[q]);
        }
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        acc[q] += __shfl_xor(acc[q], 16);
        acc[q] += __shfl_xor(acc[q], 32);
      }
      if (g == 0) {
        const double inv = LDS(O_I1 + c);
#pragma unroll
        for (int q = 0; q < NQ; ++q) LDS(O_U + c * NPAD + 16 * q + cl) = acc[q] * inv;
      }
    }
    SYNC();
  }

  // ----------------------------------------------------- H = X'X (+A'A)
  __device__ __forceinline__ void form_H(bool addAA) {
    LANE_IDS();
#pragma unroll
    for (int t = 0; t < NT; ++t) T[t] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int pp = 0; pp < NP; ++pp) {
      const int row = 4 * pp + g;
      const double cav = LDS(CA + row), cbv = LDS(CBV + row);
      const int cid = ((int)LDS(O_RC + row)) >> 2;
      double X[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q)
        X[q] = fma(cav, a_get(G[pp][q]), cbv * LDS(O_U + cid * NPAD + 16 * q + cl));
#pragma unroll
      for (int ti = 0; ti < NQ; ++ti)
#pragma unroll
        for (int tj = 0; tj <= ti; ++tj) T[tri(ti, tj)] = mfma(X[ti], X[tj], T[tri(ti, tj)]);
      if (pp % 2 == 1) SCHED_FENCE();
    }
    if (addAA) {
#pragma unroll
      for (int tm = 0; tm < MQ; ++tm)
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const int rowA = 16 * tm + g + 4 * s;
          double Aq[NQ];
#pragma unroll
          for (int q = 0; q < NQ; ++q) Aq[q] = LDS(O_A + rowA * LDA + 16 * q + cl);
#pragma unroll
          for (int ti = 0; ti < NQ; ++ti)
#pragma unroll
            for (int tj = 0; tj <= ti; ++tj) T[tri(ti, tj)] = mfma(Aq[ti], Aq[tj], T[tri(ti, tj)]);
        }
    }
#pragma unroll
    for (int ti = 0; ti < NQ; ++ti)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int R = 16 * ti + g + 4 * r, Cc = 16 * ti + cl;
        if (R == Cc && R >= n) T[tri(ti, ti)][r] = 1.0;
      }
  }

  // Symmetric Gauss-Jordan sweep of the first nact pivots of a symmetric
  // matrix held as lower tiles in C/D layout; leaves -M^-1 there.  Pivot p is
  // the Schur complement = (Cholesky diagonal)^2, so the failure test is the
  // one LAPACK potrf applies inside cholesky! (ajj <= 0 or NaN).
  //
  // Blocked by 16-pivot panels P.  The 16 single-pivot steps run only on the
  // panel slab [M_PP | Z] (Z_i = M_Pi, rows P, cols i != P), which they turn
  // into [-M_PP^-1 | M_PP^-1 Z].  The rank-1 updates the single-pivot sweep
  // would apply to every other tile are deferred: at step c the current row c
  // of Z over sqrt(d_c) is row c of W = L_PP^-1 Z, and M_OO -= W'W is applied
  // once per panel with MFMA -- the same sum of rank-1 terms (Gram form, as
  // accurate as the unblocked sweep; the explicit -M_PP^-1-based update is not).
  template <int Q>
  __device__ __forceinline__ bool sweep(d4 (&M)[Q * (Q + 1) / 2], int nact) {
    LANE_IDS();
    int step = 0;
#pragma unroll
    for (int P = 0; P < Q; ++P) {
      if (16 * P >= nact) break;
      const int cnt = (nact - 16 * P) < 16 ? (nact - 16 * P) : 16;
      d4 Z[Q], W[Q];
#pragma unroll
      for (int i = 0; i < Q; ++i) {
        W[i] = (d4){0.0, 0.0, 0.0, 0.0};
        if (i < P) Z[i] = M[tri(P, i)];
        if (i > P) Z[i] = transpose(M[tri(i, P)]);
      }
      d4& D = M[tri(P, P)];
#pragma unroll
      for (int pr = 0; pr < 4; ++pr) {
        for (int pg = 0; pg < 4; ++pg) {
          const int c = 4 * pr + pg;
          if (c >= cnt) break;
          const int cb = O_COL + (step & 1) * SH::CB;
          ++step;
          const bool lane_c = cl == c, lane_r = g == pg;
          // gather: column c of the diagonal tile, row c of every slab tile
          if (lane_c) {
#pragma unroll
            for (int r = 0; r < 4; ++r) LDS(cb + g + 4 * r) = D[r];
          }
          if (lane_r) {
            LDS(cb + 16 + 16 * P + cl) = D[pr];
#pragma unroll
            for (int i = 0; i < Q; ++i)
              if (i != P) LDS(cb + 16 + 16 * i + cl) = Z[i][pr];
          }
          SYNC();
          const double d = uni(LDS(cb + c));
          if (!(d > 0.0)) return false;
          const double rinv = recip(d);
          const double isd = recip(sqrt(d));
          double cR[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) cR[r] = LDS(cb + g + 4 * r);
          // diagonal tile: pivot row and column both from the gathered column
          // (re-symmetrised every step, which keeps the inverse a good
          // right-inverse at kappa ~ 1e10)
          {
            const double cC = LDS(cb + cl) * rinv;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const double gen = fma(-cR[r], cC, D[r]);
              const double scol = cR[r] * rinv;
              const bool iR = (r == pr) && lane_r;
              D[r] = (iR && lane_c) ? -rinv : (lane_c ? scol : (iR ? cC : gen));
            }
          }
#pragma unroll
          for (int i = 0; i < Q; ++i) {
            if (i == P) continue;
            const double rc = LDS(cb + 16 + 16 * i + cl);  // M[c][col]
            const double rs = rc * rinv;
            if (lane_r) W[i][pr] = rc * isd;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const double gen = fma(-cR[r], rs, Z[i][r]);
              Z[i][r] = (r == pr && lane_r) ? rs : gen;
            }
          }
        }
      }
      // M_OO -= W'W (lower tiles of every other block row/column)
#pragma unroll
      for (int i = 0; i < Q; ++i) {
        if (i == P) continue;
        d4 Wn;
#pragma unroll
        for (int r = 0; r < 4; ++r) Wn[r] = -W[i][r];
#pragma unroll
        for (int j = i; j < Q; ++j) {
          if (j == P) continue;
          // tile (j, i), j >= i: += W_j' (-W_i)
          d4 acc = M[tri(j, i)];
#pragma unroll
          for (int s = 0; s < 4; ++s) acc = mfma(W[j][s], Wn[s], acc);
          M[tri(j, i)] = acc;
        }
      }
#pragma unroll
      for (int i = 0; i < Q; ++i) {
        if (i < P) M[tri(P, i)] = Z[i];
        if (i > P) M[tri(i, P)] = transpose(Z[i]);
      }
    }
    return true;
  }

  __device__ __forceinline__ d4 transpose(d4 t) {
    LANE_IDS();
    SYNC();
#pragma unroll
    for (int r = 0; r < 4; ++r) LDS(O_TB + (g + 4 * r) * 17 + cl) = t[r];
    SYNC();
    d4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = LDS(O_TB + cl * 17 + g + 4 * r);
    return o;
  }

  __device__ __forceinline__ void dump_sym(double* out) {
#pragma unroll
    for (int ti = 0; ti < NQ; ++ti)
#pragma unroll
      for (int tj = 0; tj <= ti; ++tj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int R = 16 * ti + g + 4 * r, Cc = 16 * tj + cl;
          if (R < n && Cc < n) {
            out[R * n + Cc] = T[tri(ti, tj)][r];
            if (ti != tj) out[Cc * n + R] = T[tri(ti, tj)][r];
          }
        }
  }

  // H (+A'A) -> sweep -> Li;  ALi' = Li A' (n x m);  S = A ALi';  S^-1.
  __device__ __forceinline__ int factor(bool identity, bool addAA) {
    LANE_IDS();
    STAMP(SP_OTHER);
    if (!identity) compute_U();
    STAMP(SP_U);
    form_H(addAA);
    SYNC();
    STAMP(SP_SYRK);
#ifdef SOCP_DIAG
    // diagnostic dump per problem: H, H^-1 (n x n each), lam, wbar (k each), Li A' (n x m), S (m x m)
    double* dbg = (a.dbg && a.mode == MODE_KKT) ? a.dbg + dbg_p * (int64_t)(2 * n * n + 2 * k + n * m + m * m) : nullptr;
    if (dbg) dump_sym(dbg);
#endif
    const bool okH = sweep<NQ>(T, n);
    STAMP(SP_SWEEP_H);
    if (!okH) return ST_CHOL_H;
#pragma unroll
    for (int t = 0; t < NT; ++t) T[t] = -T[t];
#ifdef SOCP_DIAG
    if (dbg) {
      dump_sym(dbg + n * n);
      for (int i = lane; i < k; i += 64) {
        dbg[2 * n * n + i] = LDS(LAM + i);
        dbg[2 * n * n + k + i] = LDS(WB + i);
      }
    }
#endif
    // S = A Li A' (densesolver.jl:49-50: ALi = A*Li, S = ALi*A'), one 16-column
    // tile of Li A' at a time: it lives only here, the solves use A (Li n0).
#pragma unroll
    for (int tq = 0; tq < MQ; ++tq) {
      d4 ALc[NQ];
#pragma unroll
      for (int ti = 0; ti < NQ; ++ti) {
        d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int tk = 0; tk < NQ; ++tk) {
          d4 Ut;
          if (tk >= ti)
            Ut = T[tri(tk, ti)];
          else
            Ut = transpose(T[tri(ti, tk)]);
#pragma unroll
          for (int s = 0; s < 4; ++s) acc = mfma(Ut[s], LDS(O_A + (16 * tq + cl) * LDA + 16 * tk + g + 4 * s), acc);
        }
        ALc[ti] = acc;
      }
#ifdef SOCP_DIAG
      if (dbg) {
        double* dA = dbg + 2 * n * n + 2 * k;
#pragma unroll
        for (int ti = 0; ti < NQ; ++ti)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int R = 16 * ti + g + 4 * r, Cc = 16 * tq + cl;
            if (R < n && Cc < m) dA[R * m + Cc] = ALc[ti][r];
          }
      }
#endif
#pragma unroll
      for (int tm = tq; tm < MQ; ++tm) {
        d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int tk = 0; tk < NQ; ++tk)
#pragma unroll
          for (int s = 0; s < 4; ++s) acc = mfma(LDS(O_A + (16 * tm + cl) * LDA + 16 * tk + g + 4 * s), ALc[tk][s], acc);
        Sv[tri(tm, tq)] = acc;
      }
    }
#pragma unroll
    for (int tm = 0; tm < MQ; ++tm)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int R = 16 * tm + g + 4 * r, Cc = 16 * tm + cl;
        if (R == Cc && R >= m) Sv[tri(tm, tm)][r] = 1.0;
      }
#ifdef SOCP_DIAG
    if (dbg) {
      double* dS = dbg + 2 * n * n + 2 * k + n * m;
#pragma unroll
      for (int tm = 0; tm < MQ; ++tm)
#pragma unroll
        for (int tq = 0; tq <= tm; ++tq)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int R = 16 * tm + g + 4 * r, Cc = 16 * tq + cl;
            if (R < m && Cc < m) dS[R * m + Cc] = Sv[tri(tm, tq)][r];
          }
    }
#endif
    SYNC();
    const bool okS = sweep<MQ>(Sv, m);
    STAMP(SP_SCHUR);
    if (!okS) return ST_CHOL_S;
#pragma unroll
    for (int t = 0; t < MT; ++t) Sv[t] = -Sv[t];
    return 0;
  }

  // out = M*v for a symmetric matrix stored as lower tiles (C/D layout).
  // Lower part: per tile row, reduce over the 16 column lanes; strictly upper
  // part (transposed off-diagonal tiles): reduce over the 4 row groups.
  template <int Q>
  __device__ __forceinline__ void symv(const d4 (&M)[Q * (Q + 1) / 2], int vin, int vout) {
    LANE_IDS();
    double vc[Q], P2[Q];
#pragma unroll
    for (int t = 0; t < Q; ++t) {
      vc[t] = LDS(vin + 16 * t + cl);
      P2[t] = 0.0;
    }
    double P1row[Q];
#pragma unroll
    for (int ti = 0; ti < Q; ++ti) {
      double vr[4], P1[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        vr[r] = LDS(vin + 16 * ti + g + 4 * r);
        double acc = 0.0;
#pragma unroll
        for (int tj = 0; tj <= ti; ++tj) acc = fma(M[tri(ti, tj)][r], vc[tj], acc);
        P1[r] = acc;
      }
#pragma unroll
      for (int tj = 0; tj < ti; ++tj)
#pragma unroll
        for (int r = 0; r < 4; ++r) P2[tj] = fma(M[tri(ti, tj)][r], vr[r], P2[tj]);
      int base = 0;
      rs16<4, 8>(P1, cl, base);  // one value per lane: row 16ti + g + 4*base
      P1row[ti] = P1[0] + 0.0 * base;
      // stash the row index in base via the lane's own cl bits (see write below)
    }
#pragma unroll
    for (int t = 0; t < Q; ++t) {
      P2[t] += __shfl_xor(P2[t], 16);
      P2[t] += __shfl_xor(P2[t], 32);
    }
    SYNC();
    {
      // rs16<4,8>: bit 8 of cl picks entries 2-3, bit 4 picks the odd one; masks
      // 2 and 1 are all-reduce steps, so the lane holds entry (cl>>3&1)*2 + (cl>>2&1)
      const int r = ((cl >> 3) & 1) * 2 + ((cl >> 2) & 1);
#pragma unroll
      for (int ti = 0; ti < Q; ++ti) LDS(vout + 16 * ti + g + 4 * r) = P1row[ti];
    }
    SYNC();
    if (g == 0) {
#pragma unroll
      for (int t = 0; t < Q; ++t) LDS(vout + 16 * t + cl) += P2[t];
    }
    SYNC();
  }

  // out[row] = (G u)[row] + add1[row] - add2[row] for rows < k (u in column layout).
  // Rows are reduced over the 16 column lanes in chunks of up to 8 row-steps.
  template <int P0, int CH>
  __device__ __forceinline__ void gemv_G_chunk(const double (&uq)[NQ], int add1, int add2, int out) {
    LANE_IDS();
    double P[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      double acc = 0.0;
#pragma unroll
      for (int q = 0; q < NQ; ++q) acc = fma(a_get(G[P0 + j][q]), uq[q], acc);
      P[j] = acc;
    }
    int base = 0;
    rs16<CH, 8>(P, cl, base);
    constexpr int CF = RSCount<CH, 8>::value;
#pragma unroll
    for (int j = 0; j < CF; ++j) {
      const int row = 4 * (P0 + base + j) + g;
      if (row < k) {
        double v = P[j];
        if (add1 >= 0) v = v + LDS(add1 + row);
        v = v - LDS(add2 + row);
        LDS(out + row) = v;
      }
    }
    if constexpr (P0 + CH < NP) {
      constexpr int NXT = (NP - P0 - CH) < 8 ? (NP - P0 - CH) : 8;
      gemv_G_chunk<P0 + CH, NXT>(uq, add1, add2, out);
    }
  }
  __device__ __forceinline__ void gemv_G(int u, int add1, int add2, int out) {
    LANE_IDS();
    double uq[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) uq[q] = LDS(u + 16 * q + cl);
    gemv_G_chunk<0, (NP < 8 ? NP : 8)>(uq, add1, add2, out);
    SYNC();
  }

  // acc[q] (all lanes) = (G' v)[16q+cl]
  __device__ __forceinline__ void gemv_Gt(int v, double (&acc)[NQ]) {
    LANE_IDS();
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = 0.0;
#pragma unroll
    for (int pp = 0; pp < NP; ++pp) {
      const double vp = LDS(v + 4 * pp + g);
#pragma unroll
      for (int q = 0; q < NQ; ++q) acc[q] = fma(a_get(G[pp][q]), vp, acc[q]);
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      acc[q] += __shfl_xor(acc[q], 16);
      acc[q] += __shfl_xor(acc[q], 32);
    }
  }

  // acc[q] (all lanes) = (A' v)[16q+cl]: rows split over the 4 lane groups
  __device__ __forceinline__ void At_mv(int v, double (&acc)[NQ]) {
    LANE_IDS();
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = 0.0;
#pragma unroll
    for (int s = 0; s < MQ * 4; ++s) {
      const int i = g + 4 * s;
      const double vi = LDS(v + i);
#pragma unroll
      for (int q = 0; q < NQ; ++q) acc[q] = fma(LDS(O_A + i * LDA + 16 * q + cl), vi, acc[q]);
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      acc[q] += __shfl_xor(acc[q], 16);
      acc[q] += __shfl_xor(acc[q], 32);
    }
  }
  // out[i] = (A u)[i] - sub[i] for i < m (columns split over the 4 lane groups);
  // returns sum of out[i]^2 on lanes g == 0
  __device__ __forceinline__ double A_mv(int u, int sub, int out) {
    LANE_IDS();
    double sq = 0.0;
#pragma unroll
    for (int tm = 0; tm < MQ; ++tm) {
      const int i = 16 * tm + cl;
      double acc = 0.0;
#pragma unroll
      for (int t = 0; t < NQ * 4; ++t) acc = fma(LDS(O_A + i * LDA + g + 4 * t), LDS(u + g + 4 * t), acc);
      acc += __shfl_xor(acc, 16);
      acc += __shfl_xor(acc, 32);
      if (g == 0 && i < m) {
        const double v = acc - LDS(sub + i);
        LDS(out + i) = v;
        sq = fma(v, v, sq);
      }
    }
    return sq;
  }

  // rd = A'y + G'z + c, rp = Ax - b, rz = Gx + s - h (solver.jl:109-118)
  __device__ __forceinline__ void residuals(double& nd, double& np_, double& gap) {
    LANE_IDS();
    double acc[NQ], at[NQ];
    gemv_Gt(Z_, acc);
    At_mv(Y_, at);
    double d2 = 0.0, zs = 0.0;
    if (g == 0) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int j = 16 * q + cl;
        if (j < n) {
          const double v = (at[q] + acc[q]) + LDS(C_ + j);
          LDS(RD + j) = v;
          d2 = fma(v, v, d2);
        }
      }
    }
    const double p2 = A_mv(X_, B_, RP);
    gemv_G(X_, S_, H_, DZ);
    for (int i = lane; i < k; i += 64) zs += LDS(Z_ + i) * LDS(S_ + i);
    nd = sqrt(wsum(d2));
    np_ = sqrt(wsum(p2));
    gap = wsum(zs);
  }

  // The matrix part of solve_kkt(::DenseSolver) (densesolver.jl:66-85), between
  // the cone ops: n0 = GWiWi*k2 + dx (+A'dy if sing); m0 = ALi*n0 - dy, taken as
  // A*(Li*n0) - dy; cy = S^-1 m0; m0 = sing ? dy - cy : -cy (init: -cy);
  // n0 += A'm0; cx = Li n0; k1 = G cx - k2.   In: RD RP T2(=W^-2 k2) K2.  Out: RX RY K1.
  __device__ __forceinline__ void solve_matrix_part(bool init) {
    LANE_IDS();
    {
      double acc[NQ], at[NQ];
      gemv_Gt(T2, acc);
      if (sing) At_mv(RP, at);
      if (g == 0) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          const int j = 16 * q + cl;
          double v = acc[q] + LDS(RD + j);
          if (sing) v = v + at[q];
          LDS(N0 + j) = v;
        }
      }
    }
    SYNC();
    symv<NQ>(T, N0, TN);   // Li n0
    A_mv(TN, RP, M0);      // m0 = A Li n0 - dy
    SYNC();
    symv<MQ>(Sv, M0, RY);  // cy = S^-1 m0
    if (lane < m) LDS(M0 + lane) = (sing && !init) ? LDS(RP + lane) - LDS(RY + lane) : -LDS(RY + lane);
    SYNC();
    {
      double at[NQ];
      At_mv(M0, at);
      if (g == 0) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) LDS(N0 + 16 * q + cl) = LDS(N0 + 16 * q + cl) + at[q];
      }
    }
    SYNC();
    symv<NQ>(T, N0, RX);   // cx = Li n0
    gemv_G(RX, -1, K2, K1);
  }

  // ------------------------------------------------------------- driver
  // solve_socp (solver.jl:40-153) as a micro-phase loop; solve_kkt
  // (densesolver.jl:54-90) is phases MP_S0..MP_S7, returning to `ret`.
  __device__ __forceinline__ void run(int64_t p) {
    STAMP(SP_LOAD);
    dbg_p = p;
    int status = ST_MAXIT, iters = 0, it = 0;
    double nd = NAN, np_ = NAN, gap = NAN;
    double sig = 0.0, mu_ipm = 0.0, tstep = 0.0;
    bool fac_ident = false, fac_aa = false, dom_step = false;
    int fret = 0, ret = 0, fst = 0;
    int after_singtest;
    VopResult vr = {0.0, 0.0, 0};
    if (a.mode == MODE_KKT) {
      for (int i = lane; i < k; i += 64) {
        LDS(S_ + i) = a.s[p * k + i];
        LDS(Z_ + i) = a.z[p * k + i];
        LDS(DZ + i) = a.dz[p * k + i];
        LDS(DS + i) = a.ds[p * k + i];
      }
      for (int j = lane; j < n; j += 64) LDS(RD + j) = a.dx[p * n + j];
      for (int i = lane; i < m; i += 64) LDS(RP + i) = a.dy[p * m + i];
      after_singtest = MP_KKT;
    } else if (a.flags & F_WARM) {
      for (int j = lane; j < n; j += 64) LDS(X_ + j) = a.x[p * n + j];
      for (int i = lane; i < m; i += 64) LDS(Y_ + i) = a.y[p * m + i];
      for (int i = lane; i < k; i += 64) {
        LDS(Z_ + i) = a.z[p * k + i];
        LDS(S_ + i) = a.s[p * k + i];
      }
      after_singtest = MP_ITER;
    } else {
      after_singtest = MP_INIT;
    }
    SYNC();
    int phase;
    if (a.sing) {
      sing = uni((int)a.sing[p]) != 0;
      phase = after_singtest;
    } else {
      sing = false;
      phase = MP_SINGTEST;
    }
    bool done = false;
    while (!done) {
      LANE_IDS();
      int op = -1, va = 0, vb = 0, vo1 = 0, vo2 = 0;
      int next = phase;
      switch (phase) {
        case MP_SINGTEST:  // Problem's `sing` (Socp.jl:49-56): is G'G positive definite?
          scaling_identity();
          fac_ident = true;
          fac_aa = false;
          fret = MP_SINGTEST_POST;
          next = MP_FACTOR;
          break;
        case MP_SINGTEST_POST:
          sing = (fst == ST_CHOL_H);
          next = after_singtest;
          break;
        case MP_FACTOR:  // setup_iter (densesolver.jl:41-52)
          fst = factor(fac_ident, fac_aa);
          if (fst && fret != MP_SINGTEST_POST) {
            status = fst;
            done = true;
          }
          next = fret;
          break;
        case MP_INIT:  // initial point: the KKT system with W = I (solver.jl:68-84)
          scaling_identity();
          fac_ident = true;
          fac_aa = sing;
          fret = MP_INIT_RHS;
          next = MP_FACTOR;
          break;
        case MP_INIT_RHS:
          for (int j = lane; j < n; j += 64) LDS(RD + j) = -LDS(C_ + j);
          for (int i = lane; i < m; i += 64) LDS(RP + i) = LDS(B_ + i);
          for (int i = lane; i < k; i += 64) {
            LDS(DZ + i) = LDS(H_ + i);
            LDS(DS + i) = 0.0;
          }
          SYNC();
          ret = MP_INIT_POST;
          next = MP_S0;
          break;
        case MP_INIT_POST:
          op = VOP_MAXSTEP;
          va = RZ;
          next = MP_INIT_SHIFT;
          break;
        case MP_INIT_SHIFT: {  // cone shift (solver.jl:86-104)
          const double alphp = vr.r0, alphd = vr.r1;  // max_step(-iz), max_step(iz)
          for (int j = lane; j < n; j += 64) LDS(X_ + j) = LDS(RX + j);
          for (int i = lane; i < m; i += 64) LDS(Y_ + i) = LDS(RY + i);
          for (int i = lane; i < k; i += 64) {
            const double iz = LDS(RZ + i), e = e_of(i);
            LDS(S_ + i) = (fabs(alphp) < a.init_eps) ? -iz : -iz + (1.0 + alphp) * e;
            LDS(Z_ + i) = (fabs(alphd) < a.init_eps) ? iz : iz + (1.0 + alphd) * e;
          }
          SYNC();
          next = MP_ITER;
          break;
        }
        case MP_ITER:  // residuals (solver.jl:109-118), then compute_scaling (:106)
          STAMP(SP_OTHER);
          residuals(nd, np_, gap);
          STAMP(SP_RESID);
          if (it >= a.maxit) {
            done = true;
            break;
          }
          op = VOP_SCALING;
          va = Z_;
          vb = S_;
          next = MP_ITER_B;
          break;
        case MP_ITER_B:
          if (vr.dom) {
            status = ST_DOMAIN;
            done = true;
            break;
          }
          op = VOP_VPROD;  // ds = lam o lam (solver.jl:120)
          va = LAM;
          vb = LAM;
          vo1 = DS;
          next = MP_ITER_C;
          break;
        case MP_ITER_C:
          if (nd + np_ + gap < a.tol) {  // exit test (solver.jl:122)
            status = ST_CONVERGED;
            done = true;
            break;
          }
          for (int j = lane; j < n; j += 64) LDS(RD + j) = -LDS(RD + j);
          for (int i = lane; i < m; i += 64) LDS(RP + i) = -LDS(RP + i);
          for (int i = lane; i < k; i += 64) {
            LDS(DZ + i) = -LDS(DZ + i);
            LDS(DS + i) = -LDS(DS + i);
          }
          SYNC();
          fac_ident = false;
          fac_aa = sing;
          fret = MP_S0;
          ret = MP_POST_A;
          dom_step = false;
          next = MP_FACTOR;
          break;
        case MP_KKT:
          op = VOP_SCALING;
          va = Z_;
          vb = S_;
          next = MP_KKT_B;
          break;
        case MP_KKT_B:
          if (vr.dom) {
            status = ST_DOMAIN;
            done = true;
            break;
          }
          fac_ident = false;
          fac_aa = sing;
          fret = MP_S0;
          ret = MP_KKT_POST;
          next = MP_FACTOR;
          break;
        case MP_KKT_POST:
          status = 0;
          for (int j = lane; j < n; j += 64) a.cx[p * n + j] = LDS(RX + j);
          for (int i = lane; i < m; i += 64) a.cy[p * m + i] = LDS(RY + i);
          for (int i = lane; i < k; i += 64) {
            a.cz[p * k + i] = LDS(RZ + i);
            a.cs[p * k + i] = LDS(RS + i);
          }
          done = true;
          break;
        // ------------------------------- solve_kkt (densesolver.jl:54-90)
        case MP_S0:
          STAMP(SP_OTHER);
          op = VOP_IPROD;  // k0 = lam^-1 o ds
          va = DS;
          vo1 = K0;
          next = MP_S1;
          break;
        case MP_S1:
          op = VOP_SCALE;  // k1 = W k0
          va = K0;
          vo1 = K1;
          next = MP_S2;
          break;
        case MP_S2:
          for (int i = lane; i < k; i += 64) LDS(K2 + i) = LDS(DZ + i) - LDS(K1 + i);
          SYNC();
          op = VOP_ISCALE;
          va = K2;
          vo1 = T1;
          next = MP_S3;
          break;
        case MP_S3:
          op = VOP_ISCALE;  // t2 = iWiW k2
          va = T1;
          vo1 = T2;
          next = MP_S4;
          break;
        case MP_S4:
          STAMP(SP_VOP);
          solve_matrix_part(ret == MP_INIT_POST);
          STAMP(SP_SOLVE);
          op = VOP_ISCALE;
          va = K1;
          vo1 = T1;
          next = MP_S5;
          break;
        case MP_S5:
          op = VOP_ISCALE;  // cz = iWiW k1
          va = T1;
          vo1 = RZ;
          next = MP_S6;
          break;
        case MP_S6:
          op = VOP_SCALE;  // k1 = W cz
          va = RZ;
          vo1 = K1;
          next = MP_S7;
          break;
        case MP_S7:
          for (int i = lane; i < k; i += 64) LDS(K0 + i) = LDS(K0 + i) - LDS(K1 + i);
          SYNC();
          op = VOP_SCALE;  // cs = W k0
          va = K0;
          vo1 = RS;
          next = ret;
          break;
        // ------------------- step length (solver.jl:128-134, 143-146)
        case MP_POST_A:
          STAMP(SP_VOP);
          op = VOP_PAIR;  // kt3 = W rz, kt2 = W^-1 rs
          va = RZ;
          vb = RS;
          vo1 = T1;
          vo2 = T2;
          next = MP_POST_B;
          break;
        case MP_POST_B:
          op = VOP_STEP1;
          va = T1;
          vb = T2;
          next = MP_POST_C;
          break;
        case MP_POST_C:
          dom_step = vr.dom != 0;
          op = VOP_STEP2;
          va = T1;
          vb = T2;
          next = MP_POST_D;
          break;
        case MP_POST_D: {
          if (dom_step) {
            status = ST_DOMAIN;
            done = true;
            break;
          }
          tstep = vr.r0;
          if (ret == MP_POST_A) {  // affine direction -> centering + corrector
            double kk = 0.0, ll = 0.0;
            for (int i = lane; i < k; i += 64) {
              kk += LDS(T2 + i) * LDS(T1 + i);
              ll += LDS(LAM + i) * LDS(LAM + i);
            }
            kk = wsum(kk);
            ll = wsum(ll);
            const double t = tstep;
            const double rho = 1.0 - t - t * t * kk / ll;
            const double cr = isnan(rho) ? rho : (rho < 0.0 ? 0.0 : (rho > 1.0 ? 1.0 : rho));
            sig = ipow(cr, a.sigma_exp);  // max(0,min(1,rho))^3 (solver.jl:133)
            mu_ipm = ll / a.deg;
            op = VOP_VPROD;  // kt1 = kt2 o kt3
            va = T2;
            vb = T1;
            vo1 = K0;
            next = MP_AFF_E;
          } else {  // combined direction -> step and update (solver.jl:143-150)
            const double stp = tstep * a.step;
            for (int j = lane; j < n; j += 64) LDS(X_ + j) = LDS(X_ + j) + LDS(RX + j) * stp;
            for (int i = lane; i < m; i += 64) LDS(Y_ + i) = LDS(Y_ + i) + LDS(RY + i) * stp;
            for (int i = lane; i < k; i += 64) {
              LDS(Z_ + i) = LDS(Z_ + i) + LDS(RZ + i) * stp;
              LDS(S_ + i) = LDS(S_ + i) + LDS(RS + i) * stp;
            }
            SYNC();
            STAMP(SP_STEP);
            iters = ++it;
            next = MP_ITER;
          }
          break;
        }
        case MP_AFF_E: {  // ds += sig*mu*e - kt2 o kt3; dx,dy,dz *= 1-sig (solver.jl:136-140)
          const double scf = 1.0 - sig;
          for (int i = lane; i < k; i += 64) {
            const double kt2 = sig * mu_ipm * e_of(i);
            LDS(DS + i) = LDS(DS + i) + (kt2 - LDS(K0 + i));
            LDS(DZ + i) = LDS(DZ + i) * scf;
          }
          for (int j = lane; j < n; j += 64) LDS(RD + j) = LDS(RD + j) * scf;
          for (int i = lane; i < m; i += 64) LDS(RP + i) = LDS(RP + i) * scf;
          SYNC();
          ret = MP_POST_A + 100;  // marks the combined pass
          next = MP_S0;
          break;
        }
        default:
          done = true;
          break;
      }
      if (done) break;
      op = uni(op);
      if (op >= 0) {
        vr = vop(op, uni(va), uni(vb), uni(vo1), uni(vo2));
        STAMP(SP_VOP);
      }
      // the combined-pass marker routes the end of the second solve to MP_POST_A
      phase = uni((next == MP_POST_A + 100) ? MP_POST_A : next);
    }
    if (a.mode == MODE_KKT) {
      if (lane == 0) a.status[p] = status;
      SYNC();
      STAMP(SP_STORE);
      return;
    }
    for (int j = lane; j < n; j += 64) a.x[p * n + j] = LDS(X_ + j);
    for (int i = lane; i < m; i += 64) a.y[p * m + i] = LDS(Y_ + i);
    for (int i = lane; i < k; i += 64) {
      a.z[p * k + i] = LDS(Z_ + i);
      a.s[p * k + i] = LDS(S_ + i);
    }
    if (lane == 0) {
      if (a.res) {
        a.res[3 * p + 0] = nd;
        a.res[3 * p + 1] = np_;
        a.res[3 * p + 2] = gap;
      }
      a.iters[p] = iters;
      a.status[p] = status;
    }
    SYNC();
    STAMP(SP_STORE);
#ifdef SOCP_DIAG
    if (lane == 0 && a.stamps) {
      for (int i = 0; i < NSTAMP; ++i) atomicAdd(a.stamps + i, (unsigned long long)st_acc[i]);
      atomicAdd(a.stamps + NSTAMP, (unsigned long long)iters);
    }
    for (int i = 0; i < NSTAMP; ++i) st_acc[i] = 0;
#endif
  }
};

template <int NQ, int NP, int MQ>
__global__ void __launch_bounds__(64, 1) socp_small_kernel(SmallArgs args) {
  Small<NQ, NP, MQ> S(args);
  S.init_tables();
  STAMP_START_S(S);
  while (true) {
    int p = 0;
    if (threadIdx.x == 0) p = atomicAdd(args.counter, 1);
    p = __shfl(p, 0);
    if ((int64_t)p >= args.B) break;
    S.load_problem(p);
    S.run(p);
  }
}

}  // namespace socp
