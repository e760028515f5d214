// socp_small.hpp — the register-resident batched dense SOCP IPM kernel (gfx950).
//
// One 64-lane wavefront owns one problem for its whole solve (persistent
// one-wave blocks pull problem indices from an atomic work counter).  The
// problem's G (k x n, the dominant data: 48 KiB at n=64,k=96) is loaded from
// HBM once per solve and stays in registers for every iteration, laid out as
// the B-operand fragment of v_mfma_f64_16x16x4_f64:
//     lane (g = lane>>4, cl = lane&15) holds G[4p+g][16q+cl] in G[p][q].
// Per iteration (reference solver.jl:105-151):
//   - NT scaling (scalings.jl:22-110) with per-cone segmented wave reductions;
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
// Code-size discipline: the solve, the factorisation and every cone vector
// op have exactly one instance in the kernel (phase machine + the shared
// out-of-line cone_vop), which keeps the instruction stream cache-resident.
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
  double* dbg;  // optional (KKT mode): per problem H[n*n], Li[n*n], lam[k], wb[k]
  ConeTable cones;
};

// ------------------------------------------------------------ LDS layout
// Fixed region (independent of the template shape, used by cone_vop):
enum : int {
  O_RC = 0,                  // rcode[KMAX]: cone*4 + type (0 POC, 1 SOC head, 2 SOC tail, 3 pad)
  O_COFF = O_RC + KMAX,      // cone offs[NCS]
  O_CDIM = O_COFF + NCS,     // cone dim[NCS]
  O_CKIND = O_CDIM + NCS,    // cone kind[NCS]
  O_MU = O_CKIND + NCS,      // mu per cone
  O_I1 = O_MU + NCS,         // 1/(1+wb0) per cone
  O_TOT = O_I1 + NCS,        // reduced values per cone [NCS][4]
  O_PART = O_TOT + 4 * NCS,  // per-slot partials [2][NCS][4]
  O_KV = O_PART + 8 * NCS,   // 16 k-vectors of KMAX
  O_FIXED_END = O_KV + 16 * KMAX
};
// k-vector ids
enum : int { KV_H, KV_Z, KV_S, KV_DZ, KV_DS, KV_RZ, KV_RS, KV_LAM, KV_WB, KV_CA, KV_CB, KV_K0,
             KV_K1, KV_K2, KV_T1, KV_T2 };
__host__ __device__ constexpr int kv(int id) { return O_KV + id * KMAX; }

template <int NQ, int NP, int MQ>
struct Shape {
  static constexpr int NPAD = 16 * NQ, KP = 4 * NP, MPAD = 16 * MQ, LDA = NPAD + 1;
  static constexpr int CB = (NPAD > MPAD ? NPAD : MPAD);
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
  int NPAD = 16 * NQ, MPAD = 16 * MQ, LDA = NPAD + 1, CB = NPAD > MPAD ? NPAD : MPAD;
  int total = O_FIXED_END + MPAD * LDA + 6 * NPAD + 6 * MPAD + NCS * NPAD + 2 * CB + 16 * 17;
  return (size_t)total * sizeof(double);
}

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

__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ constexpr int tri(int i, int j) { return i * (i + 1) / 2 + j; }
__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ double wmax(double v) {
#pragma unroll
  for (int o = 32; o; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ double sel4(d4 t, int r) {
  double v = t[0];
  v = (r == 1) ? t[1] : v;
  v = (r == 2) ? t[2] : v;
  v = (r == 3) ? t[3] : v;
  return v;
}

// --------------------------------------------------------- cone vector ops
enum : int { VOP_SCALE, VOP_ISCALE, VOP_PAIR, VOP_IPROD, VOP_VPROD, VOP_SCALING, VOP_STEP,
             VOP_MAXSTEP };

struct VopResult {
  double r0, r1;
  int dom;
};

// Per-cone segmented reduction of up to 3 values over the compact layout
// (element i = 64*slot + lane): inclusive Kogge-Stone scan inside each
// cone's lane range, partials per slot in LDS, totals in LDS[O_TOT + c*4+v].
// SOC segments are summed; POC segments take the max when poc_max is set.
__device__ __forceinline__ void seg_reduce3(double (&vals)[2][3], int nv, bool poc_max, int k,
                                            int nc, const int (&ci)[2], const int (&ssl)[2],
                                            const int (&sle)[2], const bool (&ismax)[2]) {
  const int lane = threadIdx.x;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    if (64 * s < k) {
      double x[3] = {vals[s][0], vals[s][1], vals[s][2]};
      const bool mx = poc_max && ismax[s];
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const bool ok = (lane - off) >= ssl[s];
#pragma unroll
        for (int v = 0; v < 3; ++v) {
          if (v < nv) {
            double y = __shfl_up(x[v], off);
            double r = mx ? fmax(x[v], y) : x[v] + y;
            x[v] = ok ? r : x[v];
          }
        }
      }
      if (lane == sle[s]) {
#pragma unroll
        for (int v = 0; v < 3; ++v) LDS(O_PART + (s * NCS + ci[s]) * 4 + v) = x[v];
      }
    }
  }
  SYNC();
  if (lane < nc) {
    const int c = lane;
    const int o = (int)LDS(O_COFF + c), d = (int)LDS(O_CDIM + c);
    const bool mx = poc_max && (int)LDS(O_CKIND + c) == POC_K;
    const int s0 = o >> 6, s1 = (o + d - 1) >> 6;
#pragma unroll
    for (int v = 0; v < 3; ++v) {
      double t = LDS(O_PART + (s0 * NCS + c) * 4 + v);
      if (s1 > s0) {
        double u = LDS(O_PART + (s1 * NCS + c) * 4 + v);
        t = mx ? fmax(t, u) : t + u;
      }
      LDS(O_TOT + c * 4 + v) = t;
    }
  }
  SYNC();
}

// One out-of-line instance for every per-cone vector operation.  a, b, o1, o2
// are LDS offsets of k-vectors.  Reference: scale!/iscale! (scalings.jl:112-173),
// iprod!/vprod! (vectors.jl:58-125), compute_scaling (scalings.jl:22-99),
// compute_step/scmax (mats.jl:30-86), max_step (mats.jl:1-28).
static __device__ __noinline__ VopResult cone_vop(int op, int a, int b, int o1, int o2, int k, int nc) {
  const int lane = threadIdx.x;
  int ci[2], kd[2], eo[2], ssl[2], sle[2];
  bool ev[2], hd[2], tail[2], poc[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int i = 64 * s + lane;
    ev[s] = i < k;
    const int code = ev[s] ? (int)LDS(O_RC + i) : 3;
    const int c = ev[s] ? (code >> 2) : 0;
    ci[s] = c;
    kd[s] = ev[s] ? (code & 3) : 3;
    hd[s] = kd[s] == 1;
    tail[s] = kd[s] == 2;
    poc[s] = kd[s] == 0;
    const int o = ev[s] ? (int)LDS(O_COFF + c) : i;
    const int d = ev[s] ? (int)LDS(O_CDIM + c) : 1;
    eo[s] = o;
    const int st = o > 64 * s ? o : 64 * s;
    const int en = (o + d) < 64 * (s + 1) ? (o + d) : 64 * (s + 1);
    ssl[s] = ev[s] ? st - 64 * s : lane;
    sle[s] = ev[s] ? en - 1 - 64 * s : -1;
  }
  const int LAM = kv(KV_LAM), WB = kv(KV_WB);
  double v[2][3];
  int nv = 1;
  bool pmax = false;
  VopResult R = {0.0, 0.0, 0};
  // ---------------- phase 1: reduction inputs
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int i = 64 * s + lane;
    v[s][0] = v[s][1] = v[s][2] = 0.0;
    if (op == VOP_SCALE || op == VOP_ISCALE) {
      v[s][0] = tail[s] ? LDS(WB + i) * LDS(a + i) : 0.0;
    } else if (op == VOP_PAIR) {
      v[s][0] = tail[s] ? LDS(WB + i) * LDS(a + i) : 0.0;
      v[s][1] = tail[s] ? LDS(WB + i) * LDS(b + i) : 0.0;
    } else if (op == VOP_IPROD) {
      const double li = LDS(LAM + i);
      v[s][0] = tail[s] ? li * li : 0.0;
      v[s][1] = tail[s] ? LDS(a + i) * li : 0.0;
    } else if (op == VOP_VPROD) {
      v[s][0] = (tail[s] || hd[s]) ? LDS(a + i) * LDS(b + i) : 0.0;
    } else if (op == VOP_SCALING) {  // a = z, b = s
      const double zi = LDS(a + i), si = LDS(b + i);
      v[s][0] = tail[s] ? zi * zi : 0.0;
      v[s][1] = tail[s] ? si * si : 0.0;
      v[s][2] = tail[s] ? zi * si : 0.0;
    } else if (op == VOP_STEP) {  // scmax(l, a), scmax(l, b)
      const double li = LDS(LAM + i);
      v[s][0] = tail[s] ? li * li : (poc[s] ? -LDS(a + i) / li : 0.0);
      v[s][1] = tail[s] ? li * LDS(a + i) : (poc[s] ? -LDS(b + i) / li : 0.0);
      v[s][2] = tail[s] ? li * LDS(b + i) : 0.0;
    } else if (op == VOP_MAXSTEP) {  // max_step(-a), max_step(a)
      const double xi = LDS(a + i);
      v[s][0] = tail[s] ? xi * xi : (poc[s] ? xi : 0.0);
      v[s][1] = poc[s] ? -xi : 0.0;
    }
  }
  if (op == VOP_PAIR || op == VOP_IPROD) nv = 2;
  if (op == VOP_SCALING || op == VOP_STEP) nv = 3;
  if (op == VOP_MAXSTEP) nv = 2;
  pmax = (op == VOP_STEP || op == VOP_MAXSTEP);
  seg_reduce3(v, nv, pmax, k, nc, ci, ssl, sle, poc);

  // ---------------- phase 2: outputs
  if (op == VOP_STEP) {
    // second round: r2s for both directions; keep the first-round POC maxima
    double av[2] = {0.0, 0.0}, r1a[2] = {0.0, 0.0}, r1b[2] = {0.0, 0.0}, pm[2];
    bool dm = false;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = 64 * s + lane;
      const int c = ci[s];
      pm[s] = poc[s] ? fmax(LDS(O_TOT + c * 4), LDS(O_TOT + c * 4 + 1)) : -INFINITY;
      v[s][0] = v[s][1] = v[s][2] = 0.0;
      if (tail[s] || hd[s]) {
        const int o = eo[s];
        const double l0 = LDS(LAM + o);
        const double ai = l0 * l0 - LDS(O_TOT + c * 4);
        dm |= ai < 0.0;
        const double aa = 1.0 / sqrt(ai);
        const double xa0 = LDS(a + o), xb0 = LDS(b + o);
        const double ra = aa * l0 * xa0 - aa * LDS(O_TOT + c * 4 + 1);
        const double rb = aa * l0 * xb0 - aa * LDS(O_TOT + c * 4 + 2);
        av[s] = aa;
        r1a[s] = ra;
        r1b[s] = rb;
        if (tail[s]) {
          const double csa = (ra + xa0) / (aa * l0 + 1.0);
          const double csb = (rb + xb0) / (aa * l0 + 1.0);
          const double li = LDS(LAM + i);
          const double qa = aa * (LDS(a + i) - csa * aa * li);
          const double qb = aa * (LDS(b + i) - csb * aa * li);
          v[s][0] = qa * qa;
          v[s][1] = qb * qb;
        }
      }
    }
    SYNC();
    seg_reduce3(v, 2, false, k, nc, ci, ssl, sle, poc);
    double best = -INFINITY;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (poc[s]) best = fmax(best, pm[s]);
      if (hd[s]) {
        const int c = ci[s];
        const double va = sqrt(LDS(O_TOT + c * 4)) - av[s] * r1a[s];
        const double vb = sqrt(LDS(O_TOT + c * 4 + 1)) - av[s] * r1b[s];
        best = fmax(best, fmax(va, vb));
      }
    }
    double t = wmax(best);
    if (isnan(t)) t = -INFINITY;
    t = fmax(t, 0.0);
    R.r0 = (t == 0.0) ? 1.0 : fmin(1.0, 1.0 / t);
    R.dom = __any(dm) ? 1 : 0;
    return R;
  }
  if (op == VOP_MAXSTEP) {
    double bm = -INFINITY, bp = -INFINITY;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = ci[s];
      if (poc[s]) {
        bm = fmax(bm, LDS(O_TOT + c * 4));
        bp = fmax(bp, LDS(O_TOT + c * 4 + 1));
      } else if (hd[s]) {
        const double nr = sqrt(LDS(O_TOT + c * 4));
        const double x0 = LDS(a + eo[s]);
        bm = fmax(bm, nr + x0);
        bp = fmax(bp, nr - x0);
      }
    }
    R.r0 = wmax(bm);
    R.r1 = wmax(bp);
    return R;
  }
  bool dm = false;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    if (!ev[s]) continue;
    const int i = 64 * s + lane, c = ci[s], o = eo[s];
    if (op == VOP_SCALE || op == VOP_ISCALE || op == VOP_PAIR) {
      const double wi = LDS(WB + i), xi = LDS(a + i);
      double r;
      if (poc[s]) {
        r = (op == VOP_ISCALE) ? (1.0 / wi) * xi : wi * xi;
      } else {
        const double mu = LDS(O_MU + c), del = LDS(O_TOT + c * 4), wb0 = LDS(WB + o),
                     x0 = LDS(a + o);
        if (op != VOP_ISCALE) {
          const double cst = x0 + del / (1.0 + wb0);
          r = hd[s] ? mu * (wb0 * x0 + del) : mu * (xi + cst * wi);
        } else {
          const double cst = -x0 + del / (1.0 + wb0);
          const double im = 1.0 / mu;
          r = hd[s] ? im * (wb0 * x0 - del) : im * (xi + cst * wi);
        }
      }
      if (op == VOP_PAIR) {
        const double x2 = LDS(b + i);
        double r2;
        if (poc[s]) {
          r2 = (1.0 / wi) * x2;
        } else {
          const double mu = LDS(O_MU + c), del = LDS(O_TOT + c * 4 + 1), wb0 = LDS(WB + o),
                       x0 = LDS(b + o);
          const double cst = -x0 + del / (1.0 + wb0);
          const double im = 1.0 / mu;
          r2 = hd[s] ? im * (wb0 * x0 - del) : im * (x2 + cst * wi);
        }
        LDS(o2 + i) = r2;
      }
      LDS(o1 + i) = r;
    } else if (op == VOP_IPROD) {
      const double vi = LDS(a + i), li = LDS(LAM + i);
      double r;
      if (poc[s]) {
        r = vi / li;
      } else {
        const double l0 = LDS(LAM + o), v0 = LDS(a + o);
        const double aa = l0 * l0 - LDS(O_TOT + c * 4);
        const double dt = LDS(O_TOT + c * 4 + 1);
        r = hd[s] ? v0 * l0 / aa - dt / aa : -(v0 * li / aa) + vi / l0 + li * dt / (l0 * aa);
      }
      LDS(o1 + i) = r;
    } else if (op == VOP_VPROD) {
      const double ui = LDS(a + i), vi = LDS(b + i);
      double r;
      if (poc[s])
        r = ui * vi;
      else
        r = hd[s] ? LDS(O_TOT + c * 4) : LDS(a + o) * vi + LDS(b + o) * ui;
      LDS(o1 + i) = r;
    } else if (op == VOP_SCALING) {
      // compute_scaling (scalings.jl:22-99) -> lam, wb, mu, 1/(1+wb0), and
      // X = W^-1 G row coefficients: X[i,:] = ca[i] G[i,:] + cb[i] U[cone(i),:]
      const double zi = LDS(a + i), si = LDS(b + i);
      double wbi, li, cai, cbi;
      if (poc[s]) {
        const double r = si / zi, pr = si * zi, ir = zi / si;
        dm |= (r < 0.0) || (pr < 0.0) || (ir < 0.0);
        wbi = sqrt(r);
        li = sqrt(pr);
        cai = sqrt(ir);
        cbi = 0.0;
      } else {
        const double z0 = LDS(a + o), s0 = LDS(b + o);
        const double onrmz = z0 * z0 - LDS(O_TOT + c * 4), onrms = s0 * s0 - LDS(O_TOT + c * 4 + 1);
        dm |= (onrmz < 0.0) || (onrms < 0.0);
        const double nrmz = sqrt(onrmz), nrms = sqrt(onrms);
        const double fz = 1.0 / nrmz, fs = 1.0 / nrms;
        const double zb0 = z0 * fz, sb0 = s0 * fs;
        const double nsum = zb0 * sb0 + LDS(O_TOT + c * 4 + 2) * fz * fs;
        const double garg = (1.0 + nsum) / 2.0;
        dm |= garg < 0.0;
        const double gamma = sqrt(garg);
        const double fg = 1.0 / (2.0 * gamma);
        const double wb0 = (sb0 + zb0) * fg;
        const double zbi = zi * fz, sbi = si * fs;
        wbi = hd[s] ? wb0 : (sbi - zbi) * fg;
        const double ratio = nrms / nrmz, prod = nrms * nrmz;
        dm |= (ratio < 0.0) || (prod < 0.0);
        const double mu = sqrt(ratio);
        const double tmv1 = sqrt(prod);
        const double mult = tmv1 / (zb0 + sb0 + 2.0 * gamma);
        li = hd[s] ? gamma * tmv1 : (sbi * (gamma + zb0) + zbi * (gamma + sb0)) * mult;
        const double im = 1.0 / mu;
        cai = hd[s] ? -im : im;
        cbi = hd[s] ? -(1.0 + wb0) * im : wbi * im;
        if (hd[s]) {
          LDS(O_MU + c) = mu;
          LDS(O_I1 + c) = 1.0 / (1.0 + wb0);
        }
      }
      LDS(WB + i) = wbi;
      LDS(LAM + i) = li;
      LDS(kv(KV_CA) + i) = cai;
      LDS(kv(KV_CB) + i) = cbi;
    }
  }
  SYNC();
  R.dom = __any(dm) ? 1 : 0;
  return R;
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

enum { P_SINGTEST, P_INIT, P_ITER, P_AFFINE, P_COMBINED, P_KKT };

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

  AD G[NP][NQ];  // AGPR-resident
  d4 T[NT];
  d4 AL[NQ * MQ];
  d4 Sv[MT];

  __device__ __forceinline__ Small(const SmallArgs& args)
      : a(args), lane(threadIdx.x), g(threadIdx.x >> 4), cl(threadIdx.x & 15),
        n(args.n), m(args.m), k(args.k), nc(args.nc) {}

  __device__ __forceinline__ VopResult vop(int op, int x, int y, int o1, int o2) {
    return cone_vop(op, x, y, o1, o2, k, nc);
  }

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
  }

  __device__ __forceinline__ void load_problem(int64_t p) {
    const double* Gp = a.G + p * (int64_t)k * n;
#pragma unroll
    for (int pp = 0; pp < NP; ++pp) {
      const int row = 4 * pp + g;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int col = 16 * q + cl;
        a_put(G[pp][q], (row < k && col < n) ? Gp[(int64_t)col * k + row] : 0.0);
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

  // U[c,:] = (sum_{i in cone c} w_i G[i,:]) / (1+wb0), w_head = -(1+wb0), w_tail = wb_i
  __device__ __forceinline__ void compute_U() {
    for (int c = 0; c < nc; ++c) {
      if ((int)LDS(O_CKIND + c) != SOC_K) continue;
      const int o = (int)LDS(O_COFF + c), d = (int)LDS(O_CDIM + c);
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
  template <int Q>
  __device__ __forceinline__ bool sweep(d4 (&M)[Q * (Q + 1) / 2], int nact) {
    for (int p = 0; p < nact; ++p) {
      const int cb = O_COL + (p & 1) * SH::CB;
      const int tp = p >> 4, pc = p & 15, pr = pc >> 2, pg = pc & 3;
#pragma unroll
      for (int ti = 0; ti < Q; ++ti)
#pragma unroll
        for (int tj = 0; tj <= ti; ++tj) {
          if (tj == tp && cl == pc) {
#pragma unroll
            for (int r = 0; r < 4; ++r) LDS(cb + 16 * ti + g + 4 * r) = M[tri(ti, tj)][r];
          }
          if (ti == tp && tj < tp && g == pg) LDS(cb + 16 * tj + cl) = sel4(M[tri(ti, tj)], pr);
        }
      SYNC();
      const double d = LDS(cb + p);
      if (!(d > 0.0)) return false;
      const double rinv = 1.0 / d;
      double cR[Q][4], cC[Q];
#pragma unroll
      for (int ti = 0; ti < Q; ++ti) {
#pragma unroll
        for (int r = 0; r < 4; ++r) cR[ti][r] = LDS(cb + 16 * ti + g + 4 * r);
        cC[ti] = LDS(cb + 16 * ti + cl) * rinv;
      }
#pragma unroll
      for (int ti = 0; ti < Q; ++ti)
#pragma unroll
        for (int tj = 0; tj <= ti; ++tj) {
          d4& t = M[tri(ti, tj)];
          if (ti == tp || tj == tp) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int R = 16 * ti + g + 4 * r, Cc = 16 * tj + cl;
              const bool iR = R == p, iC = Cc == p;
              const double gen = fma(-cR[ti][r], cC[tj], t[r]);
              // pivot row and column both come from the gathered column p:
              // re-symmetrising them every step is what keeps the sweep's
              // inverse a good right-inverse at kappa ~ 1e10.
              const double scol = cR[ti][r] * rinv;
              t[r] = (iR && iC) ? -rinv : (iC ? scol : (iR ? cC[tj] : gen));
            }
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) t[r] = fma(-cR[ti][r], cC[tj], t[r]);
          }
        }
    }
    return true;
  }

  __device__ __forceinline__ d4 transpose(d4 t) {
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
    if (!identity) compute_U();
    form_H(addAA);
    SYNC();
    double* dbg = (a.dbg && a.mode == MODE_KKT) ? a.dbg + dbg_p * (int64_t)(2 * n * n + 2 * k) : nullptr;
    if (dbg) dump_sym(dbg);
    if (!sweep<NQ>(T, n)) return ST_CHOL_H;
#pragma unroll
    for (int t = 0; t < NT; ++t) T[t] = -T[t];
    if (dbg) {
      dump_sym(dbg + n * n);
      for (int i = lane; i < k; i += 64) {
        dbg[2 * n * n + i] = LDS(LAM + i);
        dbg[2 * n * n + k + i] = LDS(WB + i);
      }
    }
#pragma unroll
    for (int ti = 0; ti < NQ; ++ti) {
      d4 acc[MQ];
#pragma unroll
      for (int tm = 0; tm < MQ; ++tm) acc[tm] = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int tk = 0; tk < NQ; ++tk) {
        d4 Ut;
        if (tk >= ti)
          Ut = T[tri(tk, ti)];
        else
          Ut = transpose(T[tri(ti, tk)]);
#pragma unroll
        for (int tm = 0; tm < MQ; ++tm)
#pragma unroll
          for (int s = 0; s < 4; ++s)
            acc[tm] = mfma(Ut[s], LDS(O_A + (16 * tm + cl) * LDA + 16 * tk + g + 4 * s), acc[tm]);
      }
#pragma unroll
      for (int tm = 0; tm < MQ; ++tm) AL[ti * MQ + tm] = acc[tm];
    }
#pragma unroll
    for (int tm = 0; tm < MQ; ++tm)
#pragma unroll
      for (int tq = 0; tq <= tm; ++tq) {
        d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int tk = 0; tk < NQ; ++tk)
#pragma unroll
          for (int s = 0; s < 4; ++s)
            acc = mfma(LDS(O_A + (16 * tm + cl) * LDA + 16 * tk + g + 4 * s), AL[tk * MQ + tq][s], acc);
        Sv[tri(tm, tq)] = acc;
      }
#pragma unroll
    for (int tm = 0; tm < MQ; ++tm)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int R = 16 * tm + g + 4 * r, Cc = 16 * tm + cl;
        if (R == Cc && R >= m) Sv[tri(tm, tm)][r] = 1.0;
      }
    SYNC();
    if (!sweep<MQ>(Sv, m)) return ST_CHOL_S;
#pragma unroll
    for (int t = 0; t < MT; ++t) Sv[t] = -Sv[t];
    return 0;
  }

  // out = M*v for a symmetric matrix stored as lower tiles (C/D layout)
  template <int Q>
  __device__ __forceinline__ void symv(const d4 (&M)[Q * (Q + 1) / 2], int vin, int vout) {
    double vc[Q], vr[Q][4];
#pragma unroll
    for (int t = 0; t < Q; ++t) {
      vc[t] = LDS(vin + 16 * t + cl);
#pragma unroll
      for (int r = 0; r < 4; ++r) vr[t][r] = LDS(vin + 16 * t + g + 4 * r);
    }
    double P1[4 * Q], P2[Q];
#pragma unroll
    for (int t = 0; t < Q; ++t) P2[t] = 0.0;
#pragma unroll
    for (int ti = 0; ti < Q; ++ti)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double acc = 0.0;
#pragma unroll
        for (int tj = 0; tj <= ti; ++tj) acc = fma(M[tri(ti, tj)][r], vc[tj], acc);
        P1[ti * 4 + r] = acc;
      }
#pragma unroll
    for (int ti = 0; ti < Q; ++ti)
#pragma unroll
      for (int tj = 0; tj < ti; ++tj)
#pragma unroll
        for (int r = 0; r < 4; ++r) P2[tj] = fma(M[tri(ti, tj)][r], vr[ti][r], P2[tj]);
    int base = 0;
    rs16<4 * Q, 8>(P1, cl, base);
    constexpr int CF = RSCount<4 * Q, 8>::value;
#pragma unroll
    for (int t = 0; t < Q; ++t) {
      P2[t] += __shfl_xor(P2[t], 16);
      P2[t] += __shfl_xor(P2[t], 32);
    }
    SYNC();
#pragma unroll
    for (int j = 0; j < CF; ++j) {
      const int idx = base + j;
      LDS(vout + 16 * (idx >> 2) + g + 4 * (idx & 3)) = P1[j];
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
    double uq[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) uq[q] = LDS(u + 16 * q + cl);
    gemv_G_chunk<0, (NP < 8 ? NP : 8)>(uq, add1, add2, out);
    SYNC();
  }

  // acc[q] (all lanes) = (G' v)[16q+cl]
  __device__ __forceinline__ void gemv_Gt(int v, double (&acc)[NQ]) {
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

  __device__ __forceinline__ double At_times(int v, int j) {
    double acc = 0.0;
    for (int r = 0; r < m; ++r) acc = fma(LDS(O_A + r * LDA + j), LDS(v + r), acc);
    return acc;
  }
  __device__ __forceinline__ double A_times(int v, int i) {
    double acc = 0.0;
    for (int j = 0; j < n; ++j) acc = fma(LDS(O_A + i * LDA + j), LDS(v + j), acc);
    return acc;
  }

  // ------------------------------------------------------------ KKT solve
  // solve_kkt(::DenseSolver) (densesolver.jl:54-90) for (RD,RP,DZ,DS) ->
  // (RX,RY,RZ,RS).  init selects m0 = -cy (exact elimination) for the W = I
  // initial-point system; otherwise the reference's sing branch is kept.
  __device__ __forceinline__ void solve(bool init) {
    vop(VOP_IPROD, DS, 0, K0, 0);              // k0 = lam^-1 o ds
    vop(VOP_SCALE, K0, 0, K1, 0);              // k1 = W k0
    for (int i = lane; i < k; i += 64) LDS(K2 + i) = LDS(DZ + i) - LDS(K1 + i);
    SYNC();
    vop(VOP_ISCALE, K2, 0, T1, 0);
    vop(VOP_ISCALE, T1, 0, T2, 0);             // t2 = iWiW k2
    double acc[NQ];
    gemv_Gt(T2, acc);                          // GWiWi*k2 = G'(W^-2 k2)
    if (g == 0) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) LDS(TN + 16 * q + cl) = acc[q];
    }
    SYNC();
    if (lane < n) {
      double v = LDS(TN + lane) + LDS(RD + lane);
      if (sing) v = v + At_times(RP, lane);
      LDS(N0 + lane) = v;
    }
    SYNC();
    {  // m0 = ALi*n0 - dy
      double vr[NQ][4];
#pragma unroll
      for (int t = 0; t < NQ; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) vr[t][r] = LDS(N0 + 16 * t + g + 4 * r);
#pragma unroll
      for (int tm = 0; tm < MQ; ++tm) {
        double pacc = 0.0;
#pragma unroll
        for (int ti = 0; ti < NQ; ++ti)
#pragma unroll
          for (int r = 0; r < 4; ++r) pacc = fma(AL[ti * MQ + tm][r], vr[ti][r], pacc);
        pacc += __shfl_xor(pacc, 16);
        pacc += __shfl_xor(pacc, 32);
        const int i = 16 * tm + cl;
        if (g == 0 && i < m) LDS(M0 + i) = pacc - LDS(RP + i);
      }
    }
    SYNC();
    symv<MQ>(Sv, M0, RY);                      // cy = S^-1 m0
    if (lane < m) LDS(M0 + lane) = (sing && !init) ? LDS(RP + lane) - LDS(RY + lane) : -LDS(RY + lane);
    SYNC();
    if (lane < n) LDS(N0 + lane) = LDS(N0 + lane) + At_times(M0, lane);
    SYNC();
    symv<NQ>(T, N0, RX);                       // cx = Li n0
    gemv_G(RX, -1, K2, K1);                    // k1 = G cx - k2
    vop(VOP_ISCALE, K1, 0, T1, 0);
    vop(VOP_ISCALE, T1, 0, RZ, 0);             // cz = iWiW k1
    vop(VOP_SCALE, RZ, 0, K1, 0);              // k1 = W cz
    for (int i = lane; i < k; i += 64) LDS(K0 + i) = LDS(K0 + i) - LDS(K1 + i);
    SYNC();
    vop(VOP_SCALE, K0, 0, RS, 0);              // cs = W k0
  }

  // rd = A'y + G'z + c, rp = Ax - b, rz = Gx + s - h (solver.jl:109-118)
  __device__ __forceinline__ void residuals(double& nd, double& np_, double& gap) {
    double acc[NQ];
    gemv_Gt(Z_, acc);
    if (g == 0) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) LDS(TN + 16 * q + cl) = acc[q];
    }
    SYNC();
    double d2 = 0.0, p2 = 0.0, zs = 0.0;
    if (lane < n) {
      const double v = At_times(Y_, lane) + LDS(TN + lane) + LDS(C_ + lane);
      LDS(RD + lane) = v;
      d2 = v * v;
    }
    if (lane < m) {
      const double v = A_times(X_, lane) - LDS(B_ + lane);
      LDS(RP + lane) = v;
      p2 = v * v;
    }
    gemv_G(X_, S_, H_, DZ);
    for (int i = lane; i < k; i += 64) zs += LDS(Z_ + i) * LDS(S_ + i);
    nd = sqrt(wsum(d2));
    np_ = sqrt(wsum(p2));
    gap = wsum(zs);
  }

  // ------------------------------------------------------------- driver
  __device__ __forceinline__ void run(int64_t p) {
    dbg_p = p;
    int status = ST_MAXIT, iters = 0, it = 0;
    double nd = NAN, np_ = NAN, gap = NAN;
    double sig = 0.0, mu_ipm = 0.0;
    int phase;
    int after_singtest;
    if (a.mode == MODE_KKT) {
      for (int i = lane; i < k; i += 64) {
        LDS(S_ + i) = a.s[p * k + i];
        LDS(Z_ + i) = a.z[p * k + i];
        LDS(DZ + i) = a.dz[p * k + i];
        LDS(DS + i) = a.ds[p * k + i];
      }
      for (int j = lane; j < n; j += 64) LDS(RD + j) = a.dx[p * n + j];
      for (int i = lane; i < m; i += 64) LDS(RP + i) = a.dy[p * m + i];
      after_singtest = P_KKT;
    } else if (a.flags & F_WARM) {
      for (int j = lane; j < n; j += 64) LDS(X_ + j) = a.x[p * n + j];
      for (int i = lane; i < m; i += 64) LDS(Y_ + i) = a.y[p * m + i];
      for (int i = lane; i < k; i += 64) {
        LDS(Z_ + i) = a.z[p * k + i];
        LDS(S_ + i) = a.s[p * k + i];
      }
      after_singtest = P_ITER;
    } else {
      after_singtest = P_INIT;
    }
    SYNC();
    if (a.sing) {
      sing = a.sing[p] != 0;
      phase = after_singtest;
    } else {
      sing = false;
      phase = P_SINGTEST;
    }
    while (true) {
      // ------------------------------------------------ stage 1: factor
      if (phase != P_COMBINED) {
        bool ident = phase == P_SINGTEST || phase == P_INIT;
        if (ident) {
          scaling_identity();
        } else {
          if (phase == P_ITER) {
            residuals(nd, np_, gap);
            if (it >= a.maxit) break;
          }
          VopResult sr = vop(VOP_SCALING, Z_, S_, 0, 0);
          if (sr.dom) {
            status = ST_DOMAIN;
            break;
          }
          if (phase == P_ITER) {
            vop(VOP_VPROD, LAM, LAM, DS, 0);     // ds = lam o lam
            if (nd + np_ + gap < a.tol) {
              status = ST_CONVERGED;
              break;
            }
            for (int j = lane; j < n; j += 64) LDS(RD + j) = -LDS(RD + j);
            for (int i = lane; i < m; i += 64) LDS(RP + i) = -LDS(RP + i);
            for (int i = lane; i < k; i += 64) {
              LDS(DZ + i) = -LDS(DZ + i);
              LDS(DS + i) = -LDS(DS + i);
            }
            SYNC();
          }
        }
        const int st = factor(ident, phase == P_SINGTEST ? false : sing);
        if (phase == P_SINGTEST) {
          sing = (st == ST_CHOL_H);
          phase = after_singtest;
          continue;
        }
        if (st) {
          status = st;
          break;
        }
        if (phase == P_INIT) {
          for (int j = lane; j < n; j += 64) LDS(RD + j) = -LDS(C_ + j);
          for (int i = lane; i < m; i += 64) LDS(RP + i) = LDS(B_ + i);
          for (int i = lane; i < k; i += 64) {
            LDS(DZ + i) = LDS(H_ + i);
            LDS(DS + i) = 0.0;
          }
          SYNC();
        }
        if (phase == P_ITER) phase = P_AFFINE;
      }
      // ------------------------------------------------ stage 2: solve
      solve(phase == P_INIT);
      // ------------------------------------------------ stage 3: use it
      if (phase == P_KKT) {
        status = 0;
        for (int j = lane; j < n; j += 64) a.cx[p * n + j] = LDS(RX + j);
        for (int i = lane; i < m; i += 64) a.cy[p * m + i] = LDS(RY + i);
        for (int i = lane; i < k; i += 64) {
          a.cz[p * k + i] = LDS(RZ + i);
          a.cs[p * k + i] = LDS(RS + i);
        }
        break;
      }
      if (phase == P_INIT) {
        // initial point and cone shift (solver.jl:84-104)
        const VopResult ms = vop(VOP_MAXSTEP, RZ, 0, 0, 0);
        const double alphp = ms.r0, alphd = ms.r1;  // max_step(-iz), max_step(iz)
        for (int j = lane; j < n; j += 64) LDS(X_ + j) = LDS(RX + j);
        for (int i = lane; i < m; i += 64) LDS(Y_ + i) = LDS(RY + i);
        for (int i = lane; i < k; i += 64) {
          const double iz = LDS(RZ + i), e = e_of(i);
          LDS(S_ + i) = (fabs(alphp) < a.init_eps) ? -iz : -iz + (1.0 + alphp) * e;
          LDS(Z_ + i) = (fabs(alphd) < a.init_eps) ? iz : iz + (1.0 + alphd) * e;
        }
        SYNC();
        phase = P_ITER;
        continue;
      }
      vop(VOP_PAIR, RZ, RS, T1, T2);           // kt3 = W rz, kt2 = W^-1 rs
      const VopResult sr = vop(VOP_STEP, T1, T2, 0, 0);
      if (sr.dom) {
        status = ST_DOMAIN;
        break;
      }
      const double t = sr.r0;
      if (phase == P_AFFINE) {
        double kk = 0.0, ll = 0.0;
        for (int i = lane; i < k; i += 64) {
          kk += LDS(T2 + i) * LDS(T1 + i);
          ll += LDS(LAM + i) * LDS(LAM + i);
        }
        kk = wsum(kk);
        ll = wsum(ll);
        const double rho = 1.0 - t - t * t * kk / ll;
        const double cr = isnan(rho) ? rho : (rho < 0.0 ? 0.0 : (rho > 1.0 ? 1.0 : rho));
        sig = (a.sigma_exp == 3) ? cr * cr * cr : pow(cr, (double)a.sigma_exp);
        mu_ipm = ll / a.deg;
        const double scf = 1.0 - sig;
        vop(VOP_VPROD, T2, T1, K0, 0);         // kt1 = kt2 o kt3
        for (int i = lane; i < k; i += 64) {
          const double kt2 = sig * mu_ipm * e_of(i);
          LDS(DS + i) = LDS(DS + i) + (kt2 - LDS(K0 + i));
          LDS(DZ + i) = LDS(DZ + i) * scf;
        }
        for (int j = lane; j < n; j += 64) LDS(RD + j) = LDS(RD + j) * scf;
        for (int i = lane; i < m; i += 64) LDS(RP + i) = LDS(RP + i) * scf;
        SYNC();
        phase = P_COMBINED;
        continue;
      }
      // P_COMBINED: step and update (solver.jl:143-150)
      const double stp = t * a.step;
      for (int j = lane; j < n; j += 64) LDS(X_ + j) = LDS(X_ + j) + LDS(RX + j) * stp;
      for (int i = lane; i < m; i += 64) LDS(Y_ + i) = LDS(Y_ + i) + LDS(RY + i) * stp;
      for (int i = lane; i < k; i += 64) {
        LDS(Z_ + i) = LDS(Z_ + i) + LDS(RZ + i) * stp;
        LDS(S_ + i) = LDS(S_ + i) + LDS(RS + i) * stp;
      }
      SYNC();
      iters = ++it;
      phase = P_ITER;
    }
    if (a.mode == MODE_KKT) {
      if (lane == 0) a.status[p] = status;
      SYNC();
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
  }
};

template <int NQ, int NP, int MQ>
__global__ void __launch_bounds__(64, 1) socp_small_kernel(SmallArgs args) {
  Small<NQ, NP, MQ> S(args);
  S.init_tables();
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
