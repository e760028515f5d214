// socp_sqr.hip — the rank-update KKT plugin on gfx950: the reference's
// SqrScaling + SparseSolver (sqrscalings.jl:8-194, spsolver.jl:1-130), i.e.
// W^-2 = D + u u' - v v' per SOC cone, H = G'DG (+A'A) factored as L L', one
// rank-1 update with G'u and one downdate with G'v per SOC cone
// (modify_factors!), S = (L^-1 A')'(L^-1 A') factored, and solve_kkt by
// triangular solves.  CHOLMOD (the reference's factoriser) is replaced by a
// dense LDS-resident factor: the batch's problems are small and dense.
//
// One wavefront per problem, n, m <= 64, k <= 256, register-resident: lane i
// holds row i of H and then of its factor L in NC (= n rounded up to 16)
// VGPR pairs; nothing in the factorisation waits on a barrier or an LDS round
// trip -- pivots and pivot-column entries come from readlane.
//   setup kernel: s, z -> scaling (per cone, wave reductions); H rows
//     accumulated from G row chunks staged through LDS (broadcast reads);
//     right-looking Cholesky in registers; per SOC cone the update (G'u) and
//     the downdate (G'v) as two chains skewed by one column; L^-1 A' by
//     forward substitution, S = C'C and chol(S) in LDS; the factor record
//     (L_H, L_S, lambda, wb, mu, status) to HBM.
//   solve kernel: L rows back into registers; forward substitution local to
//     each lane, backward substitution by one all-lane reduction per row
//     (DPP + permlane swaps); cone ops per cone; G'v with a lane per column,
//     Gv with a lane per row.
#include <hip/hip_runtime.h>

#include "socp_sqr.hpp"
#include "socp_sqr_step.hpp"

namespace socp {

namespace {

// every lane gets the sum over the wavefront (DPP row rotations + row swaps)
__device__ inline double wave_sum(double v) { return cone_allreduce_rows<false>(v, 4); }

// orders one wavefront's LDS accesses across lanes (and stops the compiler
// from moving them across this point)
__device__ inline void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

// value of lane j (j wave-uniform)
__device__ inline double bcast(double v, int j) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), j);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), j);
  return __hiloint2double(hi, lo);
}

#ifdef SOCP_DIAG
// per-phase shader-clock totals of the setup kernel (thread 0 of each
// workgroup, after the phase's barrier), summed over the batch
#define SQ_STAMP(i)                                                      \
  do {                                                                   \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();                   \
    if (C.lane == 0 && C.a.stamps) atomicAdd(C.a.stamps + (i), t_ - st_last); \
    st_last = t_;                                                        \
  } while (0)
#else
#define SQ_STAMP(i) do {} while (0)
#endif

struct Ctx {
  const SqrArgs& a;
  const SqrLayout& L;
  double* lds;
  int lane;
};

// ------------------------------------------------------------- cone ops
// scale! (inv = false) / iscale! (inv = true) of one cone (scalings.jl:112-157)
// by one wavefront; op may alias x (every element is read before it is written).
__device__ __forceinline__ void cone_scale(const double* wb, double mu, const double* x, double* op, int o, int d,
                           int kind, bool inv, int lane) {
  wsync();
  if (kind == POC_K) {
    for (int i = o + lane; i < o + d; i += 64) op[i] = inv ? recip(wb[i]) * x[i] : wb[i] * x[i];
    return;
  }
  double part = 0.0;
  for (int i = o + 1 + lane; i < o + d; i += 64) part += wb[i] * x[i];
  const double del = wave_sum(part);
  const double x0 = x[o], w0 = wb[o];
  if (inv) {
    const double cst = (-x0 + del * recip(1.0 + w0));
    const double im = recip(mu);
    for (int i = o + 1 + lane; i < o + d; i += 64) op[i] = im * (x[i] + cst * wb[i]);
    if (lane == 0) op[o] = im * (w0 * x0 - del);
  } else {
    const double cst = (x0 + del * recip(1.0 + w0));
    for (int i = o + 1 + lane; i < o + d; i += 64) op[i] = mu * (x[i] + cst * wb[i]);
    if (lane == 0) op[o] = mu * (w0 * x0 + del);
  }
  wsync();
}

// iprod! (vectors.jl:99-125): t = lam^-1 o v of one cone, closed form of the O(d^2) loop
__device__ __forceinline__ void cone_iprod(const double* lam, const double* v, double* t, int o, int d, int kind, int lane) {
  wsync();
  if (kind == POC_K) {
    for (int i = o + lane; i < o + d; i += 64) t[i] = v[i] * recip(lam[i]);
    return;
  }
  double p1 = 0.0, p2 = 0.0;
  for (int i = o + 1 + lane; i < o + d; i += 64) {
    p1 += lam[i] * lam[i];
    p2 += v[i] * lam[i];
  }
  const double ll = wave_sum(p1), lv = wave_sum(p2);
  const double l0 = lam[o], v0 = v[o];
  const double a = l0 * l0 - ll;
  const double ia = recip(a), il0 = recip(l0), ila = recip(l0 * a);
  for (int i = o + 1 + lane; i < o + d; i += 64)
    t[i] = -v0 * lam[i] * ia + v[i] * il0 + lam[i] * lv * ila;
  if (lane == 0) t[o] = v0 * l0 * ia - lv * ia;
  wsync();
}

// ------------------------------------------------------------ scaling
// compute_scaling(::SqrScaling) (sqrscalings.jl:50-58, 66-139) of cone c
__device__ __forceinline__ void sqr_scaling_cone(Ctx& C, int c) {
  const SqrLayout& L = C.L;
  double* lds = C.lds;
  const int kind = C.a.cones.kind[c], o = C.a.cones.offs[c], d = C.a.cones.dim[c];
  const double *s = lds + L.o_s, *z = lds + L.o_z;
  double *D = lds + L.o_D, *iW = lds + L.o_iW, *u = lds + L.o_u, *v = lds + L.o_v;
  double *lam = lds + L.o_l, *wb = lds + L.o_wb;
  bool bad = false;
  if (kind == POC_K) {
    for (int i = o + C.lane; i < o + d; i += 64) {
      // one rsq of s z gives sqrt(z/s) = z q, sqrt(s z) = (s z) q, sqrt(s/z) = s q
      const double sz = s[i] * z[i], q = rsqrt_nr(sz);
      bad |= sz < 0.0;
      D[i] = z[i] * recip(s[i]);
      iW[i] = zmul(z[i], q);  // s z = 0 (a boundary iterate): q = inf, the zero factors stay 0 as in IEEE sqrt
      lam[i] = zmul(sz, q);
      wb[i] = zmul(s[i], q);
      u[i] = 0.0;
      v[i] = 0.0;
    }
    if (C.lane == 0) lds[L.o_mu + c] = 1.0;
  } else {
    double ps = 0.0, pz = 0.0;
    for (int i = o + 1 + C.lane; i < o + d; i += 64) {
      ps += s[i] * s[i];
      pz += z[i] * z[i];
    }
    const double sprod = s[o] * s[o] - wave_sum(ps), zprod = z[o] * z[o] - wave_sum(pz);
    bad |= sprod < 0.0 || zprod < 0.0;
    const double fs = rsqrt_nr(sprod), fz = rsqrt_nr(zprod);
    double pn = 0.0;
    for (int i = o + C.lane; i < o + d; i += 64) pn += (z[i] * fz) * (s[i] * fs);
    const double nsum = wave_sum(pn);
    bad |= (1.0 + nsum) < 0.0;
    const double garg = (1.0 + nsum) * 0.5, rg = rsqrt_nr(garg);
    const double gamma = garg * rg, i2g = 0.5 * rg;  // sqrt((1 + nsum) / 2), 1 / (2 gamma)
    const double s0 = s[o] * fs, z0 = z[o] * fz;
    const double wb0 = (s0 + z0) * i2g;
    double pw = 0.0;
    for (int i = o + 1 + C.lane; i < o + d; i += 64) {
      const double w = (s[i] * fs - z[i] * fz) * i2g;
      wb[i] = w;
      pw += w * w;
    }
    const double wb1sq = wave_sum(pw);
    const double q = sprod * recip(zprod);
    bad |= q < 0.0;
    const double inusq = rsqrt_nr(q), rq = q * inusq;  // 1 / sqrt(q), sqrt(q)
    const double inu = rsqrt_nr(rq), mu = rq * inu;
    const double i1 = recip(1.0 + wb0);
    const double cv = -(1.0 + wb0 + wb1sq * i1);
    const double dd = 1.0 + 2.0 * i1 + wb1sq * (i1 * i1);
    const double av = (wb0 * wb0 + wb1sq - cv * cv * wb1sq * recip(1.0 + dd * wb1sq)) * 0.5;
    const double u0a = wb0 * wb0 + wb1sq - av;
    bad |= u0a < 0.0;
    const double iu0 = rsqrt_nr(u0a), u0 = u0a * iu0;
    const double u1 = cv * iu0;
    const double v1a = cv * cv / (u0 * u0) - dd;
    bad |= v1a < 0.0;
    const double v1 = sqrt_nr(v1a);
    const double tmv1 = sqrt_nr((sprod * fs) * (zprod * fz));
    const double mult = tmv1 * recip(z0 + s0 + 2.0 * gamma);
    for (int i = o + 1 + C.lane; i < o + d; i += 64) {
      D[i] = inusq;
      iW[i] = inu;  // sqrt(1 / sqrt(q))
      const double wbv = inu * wb[i];
      u[i] = u1 * wbv;
      v[i] = v1 * wbv;
      lam[i] = ((s[i] * fs) * (gamma + z0) + (z[i] * fz) * (gamma + s0)) * mult;
    }
    if (C.lane == 0) {
      D[o] = av * inusq;
      iW[o] = sqrt_nr(fabs(av * inusq));
      u[o] = inu * u0;
      v[o] = 0.0;
      wb[o] = wb0;
      lam[o] = gamma * tmv1;
      lds[L.o_mu + c] = mu;
    }
  }
  // Julia's sqrt throws DomainError on a negative argument
  if (bad) lds[L.o_flag] = (double)SQR_DOMAIN;
}

// sum_i p[i * stride] * v[i], i < cnt, in order; the loads are issued U at
// a time so one memory latency is paid per U elements, not per element
template <int U = 8>
__device__ __forceinline__ double dot_strided(const double* p, int64_t stride, const double* v, int cnt) {
  double acc = 0.0;
  int i = 0;
  for (; i + U <= cnt; i += U) {
    double g[U];
#pragma unroll
    for (int t = 0; t < U; ++t) g[t] = p[(int64_t)(i + t) * stride];
#pragma unroll
    for (int t = 0; t < U; ++t) acc += g[t] * v[i + t];
  }
  for (; i < cnt; ++i) acc += p[(int64_t)i * stride] * v[i];
  return acc;
}

// loads in flight per lane in the solve kernel's passes over G (an HBM round
// trip per SQR_GU elements; 16: -1.3 % solve kernel time at the C2 shape)
#ifndef SQR_GU
#define SQR_GU 16
#endif

#ifndef SQR_S_MFMA
#define SQR_S_MFMA 1  // 0: S = C'C one entry per lane (dot products out of LDS)
#endif
#ifndef SQR_S_REGS
#define SQR_S_REGS 1  // 0: chol(S) in LDS for every m (m <= 16: rows of S in registers)
#endif
// 1/sqrt(x) from v_rsq_f64 refined by two Newton steps (to within an ulp or
// two; x < 0 or NaN gives NaN, which the callers' status checks catch; +-0 and
// +inf give the IEEE +-inf and 0, not the 0 * inf NaN of the refinement)
__device__ __forceinline__ double rsqrt_nr(double x) {
  const double y0 = __builtin_amdgcn_rsq(x);
  const double hx = 0.5 * x;
  double y = y0 * (1.5 - hx * y0 * y0);
  y = y * (1.5 - hx * y * y);
  return __builtin_amdgcn_class(x, kClassZeroInf) ? y0 : y;
}

// ------------------------------------------------------------ factor ops
// L y = b (forward): lane i holds row i of L in h[], b[i] in b; returns y.
template <int NC>
__device__ __forceinline__ double fwd_solve(const double (&h)[NC], double rd, int n, double b, int lane) {
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const double yj = bcast(b, j) * bcast(rd, j);
    if (lane == j) b = yj;
    if (lane > j) b -= h[j] * yj;
    __builtin_amdgcn_sched_barrier(0);
  }
  return b;
}
// L' x = y (backward): x_i = (y_i - sum_{j>i} L(j,i) x_j) / L(i,i); lane j
// holds L(j,i) in h[i] and x_j, so each row is one all-lane reduction.
template <int NC>
__device__ __forceinline__ double bwd_solve(const double (&h)[NC], double rd, int n, double y, int lane) {
#pragma unroll
  for (int i = NC - 1; i >= 0; --i) {
    const double s = wave_sum(lane > i ? h[i] * y : 0.0);
    const double xi = (bcast(y, i) - s) * bcast(rd, i);
    if (lane == i) y = xi;
    __builtin_amdgcn_sched_barrier(0);
  }
  return y;
}

// one column step of a rank-1 modification L L' + sig w w' (column j):
// r = sqrt(L_jj^2 + sig w_j^2), c = r / L_jj, s = w_j / L_jj,
// L_ij = (L_ij + sig s w_i) / c, w_i = c w_i - s L_ij (i > j).  false: r^2 <= 0.
__device__ __forceinline__ bool mod_step(double& hj, double& w, double& rd, int j, double sig, int lane) {
  const double ljj = bcast(hj, j), wj = bcast(w, j), il = bcast(rd, j);
  const double r2 = ljj * ljj + sig * wj * wj;
  const double ir = rsqrt_nr(r2), r = r2 * ir;
  const double cc = r * il, sn = wj * il, icc = ljj * ir;
  if (lane == j) {
    hj = r;
    rd = ir;
  } else if (lane > j) {
    const double lij = (hj + sig * sn * w) * icc;
    hj = lij;
    w = cc * w - sn * lij;
  }
  return r2 > 0.0;
}

// chol of the m x m lower triangle of Sm (column-major, ld) by one wavefront
// in LDS (m <= 64: one row per lane); 1/diag -> rdg[]; false at a pivot <= 0
__device__ __forceinline__ bool chol_lds(double* Sm, int ld, int m, double* rdg, int lane) {
  for (int j = 0; j < m; ++j) {
    wsync();
    const double djj = Sm[j * ld + j];
    if (!(djj > 0.0)) return false;
    const double ir = rsqrt_nr(djj), r = djj * ir;
    if (lane == j) {
      Sm[j * ld + j] = r;
      rdg[j] = ir;
    }
    if (lane > j && lane < m) Sm[j * ld + lane] *= ir;
    wsync();
    if (lane > j && lane < m) {
      const double lij = Sm[j * ld + lane];
      for (int l = j + 1; l <= lane; ++l) Sm[l * ld + lane] -= lij * Sm[j * ld + l];
    }
  }
  wsync();
  return true;
}
// S^-1 b by one wavefront against chol_lds's factor; b one value per lane
__device__ __forceinline__ double chol_solve_lds(const double* Sm, int ld, const double* rdg, int m, double b, int lane) {
  for (int j = 0; j < m; ++j) {
    const double xj = bcast(b, j) * rdg[j];
    if (lane == j) b = xj;
    if (lane > j && lane < m) b -= Sm[j * ld + lane] * xj;
  }
  for (int j = m - 1; j >= 0; --j) {
    const double xj = bcast(b, j) * rdg[j];
    if (lane == j) b = xj;
    if (lane < j) b -= Sm[lane * ld + j] * xj;
  }
  return b;
}

// -------------------------------------------------------- setup kernel
template <int NC>
__device__ __forceinline__ void setup_problem(Ctx& C, int64_t p) {
  const SqrArgs& a = C.a;
  const SqrLayout& L = C.L;
  double* lds = C.lds;
  const int lane = C.lane;
  const int n = a.n, m = a.m, k = a.k, nc = a.nc;
  const double* G = a.G + p * (int64_t)k * n;
  const double* A = m ? a.A + p * (int64_t)m * n : nullptr;
  const bool sing = a.sing && a.sing[p];
  double* rec = a.rec + p * L.rec;
  if (a.active && !a.active[p]) return;
#ifdef SOCP_DIAG
  uint64_t st_last = __builtin_amdgcn_s_memtime();
#endif
  double zs = 0.0;  // s'z for the fused residuals (s, z's LDS is reused by the G'u / G'v below)
  for (int i = lane; i < k; i += 64) {
    const double si = a.s[p * k + i], zi = a.z[p * k + i];
    lds[L.o_s + i] = si;
    lds[L.o_z + i] = zi;
    lds[L.o_one + i] = 1.0;
    zs = fma(zi, si, zs);
  }
  if (lane == 0) lds[L.o_flag] = 0.0;
  wsync();
  for (int c = 0; c < nc; ++c) sqr_scaling_cone(C, c);
  wsync();
  SQ_STAMP(0);
  int status = (int)lds[L.o_flag];
  double h[NC];
  double rd = lane >= n ? 1.0 : 0.0;  // lane j: 1 / L(j,j) (1 on the identity-padded rows)
  // modify_factors!' G'u and G'v (sqrscalings.jl:160-194) of the first (up to 8)
  // SOC cones ride along the H product as one more 16-row MFMA operand (slot
  // j = 2 c' + {0: u, 1: v} of SOC cone c'), against the G row chunks already
  // staged in LDS -- no second pass over G.  The results land in the s..v
  // vectors' LDS (dead after the product: 6 KP doubles), so when they do not
  // fit, or (non-sing) a SOC row's iW is 0 (the staged rows are iW G, the
  // weights u / iW), the cones are re-read from G below.
  int c_soc = 0;
  while (c_soc < nc && a.cones.kind[c_soc] != SOC_K) ++c_soc;
  const int fslots = (nc - c_soc) < 8 ? (nc - c_soc) : 8;
  double* wuv = lds + L.o_s;  // wuv[j * n + col], j < 2 fslots: over s, z, D, iW (u, v stay for the re-read cones)
  bool fuse = status == 0 && fslots > 0 && 2 * fslots * n <= 4 * ((k + 1) / 2 * 2);
  // rows of the fused cones (contiguous): [fr0, fr1)
  const int fr0 = fslots > 0 ? a.cones.offs[c_soc] : 0;
  const int fr1 = fslots > 0 ? a.cones.offs[c_soc + fslots - 1] + a.cones.dim[c_soc + fslots - 1] : 0;
  if (fuse && !sing) {
    bool zero = false;
    for (int i = fr0 + lane; i < fr1; i += 64) zero |= !(lds[L.o_iW + i] > 0.0);
    fuse = !__any(zero);
    if (fuse) {
      wsync();
      for (int i = fr0 + lane; i < fr1; i += 64) {
        const double iw = lds[L.o_iW + i];
        lds[L.o_u + i] /= iw;
        lds[L.o_v + i] /= iw;
      }
      wsync();
    }
  }
  // fused residuals (a.fuse_resid): this lane's elements of a staged G chunk
  // are row r0 + (lane & 7) of the columns (lane >> 3) + 8 q; gz[q]
  // accumulates those columns' G'z, and each chunk's row sums of G x are
  // reduced over the eight lanes that share the row
  constexpr int PEF = SQR_KC * NC / 64;
  const bool FR = a.fuse_resid != 0;
  double xq[PEF], gz[PEF];
#pragma unroll
  for (int q = 0; q < PEF; ++q) {
    const int col = (lane >> 3) + 8 * q;
    xq[q] = (FR && col < n) ? a.ix[p * n + col] : 0.0;
    gz[q] = 0.0;
  }
  if (status == 0) {
    // ---- H = G'DG (+A'A) on f64 MFMA 16x16x4: the lower 16x16 tiles,
    // Y rows staged through LDS 8 at a time; then one LDS transpose gives each
    // lane its row of H (v_mfma_f64_16x16x4: A[i][k] / B[k][j] one f64 per
    // lane at i, j = lane & 15, k = lane >> 4; D[row][col] at col = lane & 15,
    // row = (lane >> 4) + 4 v)
    constexpr int NT = NC / 16;
    typedef double d4v __attribute__((ext_vector_type(4)));
    d4v acc[NT * (NT + 1) / 2];
#pragma unroll
    for (int t = 0; t < NT * (NT + 1) / 2; ++t) acc[t] = d4v{0.0, 0.0, 0.0, 0.0};
    d4v accx[NT];  // (w_j' G)[16X + col] of the fused G'u / G'v
#pragma unroll
    for (int t = 0; t < NT; ++t) accx[t] = d4v{0.0, 0.0, 0.0, 0.0};
    // this lane's weight slot: SOC cone c_soc + (lane & 15) / 2, u or v
    const int wslot = (lane & 15) >> 1;
    const int wo = wslot < fslots ? a.cones.offs[c_soc + wslot] : 0;
    const int we = wslot < fslots ? wo + a.cones.dim[c_soc + wslot] : 0;
    const double* wvec = lds + ((lane & 1) ? L.o_v : L.o_u);
    double *Ya = lds + L.o_X, *Yb = Ya + SQR_KC * SQR_NW;
    // non-sing: (iW G)'(iW G) (spsolver.jl:62-64); sing: G'(iWiW G) + A'A (:67-71)
    const double *fa = lds + (sing ? L.o_one : L.o_iW), *fb = lds + (sing ? L.o_D : L.o_iW);
    constexpr int PE = SQR_KC * NC / 64;  // chunk elements per lane
    for (int pass = 0; pass < (sing && m > 0 ? 2 : 1); ++pass) {
      const double* src = pass ? A : G;
      const int rows = pass ? m : k;
      // software-pipelined: chunk r0 + KC is loaded while chunk r0 is used
      double gn[PE];
#pragma unroll
      for (int q = 0; q < PE; ++q) {
        const int e = lane + 64 * q, col = e / SQR_KC, r = e % SQR_KC;
        gn[q] = (col < n && r < rows) ? src[(int64_t)col * rows + r] : 0.0;
      }
      for (int r0 = 0; r0 < rows; r0 += SQR_KC) {
        wsync();
#pragma unroll
        for (int q = 0; q < PE; ++q) {
          const int e = lane + 64 * q, col = e / SQR_KC, r = e % SQR_KC;
          const double g = gn[q];
          const bool in = r0 + r < rows;
          Ya[r * SQR_NW + col] = pass ? g : (in ? fa[r0 + r] * g : 0.0);
          Yb[r * SQR_NW + col] = pass ? g : (in ? fb[r0 + r] * g : 0.0);
        }
        if (FR && pass == 0) {
          const int row = r0 + (lane & 7);
          const double zr = row < k ? lds[L.o_z + row] : 0.0;
          double gxr = 0.0;
          static_assert(PE == PEF, "chunk elements per lane");
#pragma unroll
          for (int q = 0; q < PE; ++q) {
            gz[q] = fma(gn[q], zr, gz[q]);
            gxr = fma(gn[q], xq[q], gxr);
          }
          gxr += row_partner<8>(gxr);
          gxr = rows_sum(gxr);  // (G x)[row] in the eight lanes of the row
          if (lane < 8 && row < k) {
            const double v = gxr + lds[L.o_s + row] - a.ih[p * k + row];  // rz (solver.jl:118)
            a.odz[p * k + row] = -v;  // stored negated: the affine right-hand side (solver.jl:124)
          }
        }
#pragma unroll
        for (int q = 0; q < PE; ++q) {  // the next chunk's loads fly under this chunk's MFMAs
          const int e = lane + 64 * q, col = e / SQR_KC, r = e % SQR_KC;
          const int rn = r0 + SQR_KC + r;
          gn[q] = (col < n && rn < rows) ? src[(int64_t)col * rows + rn] : 0.0;
        }
        wsync();
#pragma unroll
        for (int s = 0; s < SQR_KC; s += 4) {
          const int rr = s + (lane >> 4), cc = lane & 15;
          double av[NT], bv[NT];
#pragma unroll
          for (int I = 0; I < NT; ++I) {
            av[I] = Ya[rr * SQR_NW + 16 * I + cc];
            bv[I] = Yb[rr * SQR_NW + 16 * I + cc];
          }
          int t = 0;
#pragma unroll
          for (int I = 0; I < NT; ++I)
#pragma unroll
            for (int J = 0; J <= I; ++J, ++t) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[I], bv[J], acc[t], 0, 0, 0);
          if (fuse && pass == 0) {
            const int row = r0 + rr;
            const double wt = (row >= wo && row < we) ? wvec[row] : 0.0;
#pragma unroll
            for (int X = 0; X < NT; ++X) accx[X] = __builtin_amdgcn_mfma_f64_16x16x4f64(wt, av[X], accx[X], 0, 0, 0);
          }
        }
      }
    }
    if (fuse) {
      wsync();  // every lane is past the product's reads of s..v
#pragma unroll
      for (int X = 0; X < NT; ++X)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int j = (lane >> 4) + 4 * v, col = 16 * X + (lane & 15);
          if (j < 2 * fslots && col < n) wuv[j * n + col] = accx[X][v];
        }
      wsync();
    }
    {
      double* T = lds + L.o_X;  // 64 x 17 staging of one 16-column block
#pragma unroll
      for (int J = 0; J < NT; ++J) {
        wsync();
#pragma unroll
        for (int I = 0; I < NT; ++I)
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int row = 16 * I + (lane >> 4) + 4 * v;
            T[row * 17 + (lane & 15)] = I >= J ? acc[I * (I + 1) / 2 + (I >= J ? J : 0)][v] : 0.0;
          }
        wsync();
#pragma unroll
        for (int c = 0; c < 16; ++c) h[16 * J + c] = T[lane * 17 + c];
      }
    }
    // rows n..NC-1 become identity rows: the padded factor is [L 0; 0 I], so
    // the unrolled column loops below need no `j < n` guards (zero-padded G
    // columns leave rows < n with zeros there)
#pragma unroll
    for (int l = 0; l < NC; ++l)
      if (lane >= n) h[l] = lane == l ? 1.0 : 0.0;
    SQ_STAMP(1);
    // ---- Cholesky, right-looking, in registers
    bool badc = false;  // a pivot <= 0 or NaN: the rest runs on NaNs, the status says so
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      if (j >= n) continue;  // one uniform branch per column (the padded pivots are 1)
      const double d = bcast(h[j], j);
      badc |= !(d > 0.0);
      const double ir = rsqrt_nr(d), r = d * ir;
      if (lane == j) {
        h[j] = r;
        rd = ir;
      } else if (lane > j) {
        h[j] *= ir;
      } else {
        h[j] = 0.0;
      }
#pragma unroll
      for (int l = j + 1; l < NC; ++l) h[l] -= h[j] * bcast(h[j], l);
      __builtin_amdgcn_sched_barrier(0);  // bounds the live ranges of straight-line code
    }
    if (badc) status = SQR_CHOL_H;
    SQ_STAMP(2);
    // ---- modify_factors! (sqrscalings.jl:160-194): per SOC cone the update
    // with G'u, then the downdate with G'v.  Two cones per sweep as four
    // chains one column apart (u1, v1, u2, v2): each column is final for the
    // earlier chains when a later one reaches it, so the result is the
    // sequential one bit for bit, and the four latency chains overlap.  The
    // SOC cones follow the POC cones (check_problem).
    int c0 = 0;
    while (c0 < nc && a.cones.kind[c0] != SOC_K) ++c0;
    for (; c0 < nc && status == 0; c0 += 2) {
      const int nch = c0 + 1 < nc ? 4 : 2;
      double w[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int slot = c0 + q - c_soc;
        if (lane < n && 2 * q < nch && fuse && slot < fslots) {  // from the fused product
          w[2 * q] = wuv[2 * slot * n + lane];
          w[2 * q + 1] = wuv[(2 * slot + 1) * n + lane];
        } else if (lane < n && 2 * q < nch) {
          const int o = a.cones.offs[c0 + q], d = a.cones.dim[c0 + q];
          for (int r = o; r < o + d; ++r) {
            const double g = G[(int64_t)lane * k + r];
            w[2 * q] += g * lds[L.o_u + r];
            w[2 * q + 1] += g * lds[L.o_v + r];
          }
        }
      }
      bool bad = false;
#pragma unroll
      for (int t = 0; t < NC + 3; ++t) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int j = t - c;
          if (j >= 0 && j < NC && (c < 2 || nch == 4)) bad |= !mod_step(h[j], w[c], rd, j, (c & 1) ? -1.0 : 1.0, lane);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (bad) status = SQR_CHOL_H;
    }
    SQ_STAMP(3);
    // ---- C = L^-1 A' (SQR_RHS right-hand sides per sweep), S = C'C, chol(S)
    if (status == 0 && m > 0) {
      double* Cm = lds + L.o_X;  // the chunk buffers are free now
      for (int q0 = 0; q0 < m; q0 += SQR_RHS) {
        double b[SQR_RHS];
#pragma unroll
        for (int t = 0; t < SQR_RHS; ++t) b[t] = (q0 + t < m && lane < n) ? A[(int64_t)lane * m + q0 + t] : 0.0;
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          const double rj = bcast(rd, j);
#pragma unroll
          for (int t = 0; t < SQR_RHS; ++t) {
            const double xj = bcast(b[t], j) * rj;
            if (lane == j) b[t] = xj;
            if (lane > j) b[t] -= h[j] * xj;
          }
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int t = 0; t < SQR_RHS; ++t)
          if (q0 + t < m && lane < n) Cm[(q0 + t) * L.ldl + lane] = b[t];
      }
      wsync();
      SQ_STAMP(4);
      double* Sm = lds + L.o_S;
#if SQR_S_MFMA
      // S = C'C by lower 16 x 16 tiles on f64 MFMA (k-steps of four rows of C)
      {
        const int g = lane >> 4, cl = lane & 15;
        const int MT = (m + 15) / 16;
        for (int I = 0; I < MT; ++I)
          for (int J = 0; J <= I; ++J) {
            d4v acc = {0.0, 0.0, 0.0, 0.0};
            const int ci = 16 * I + cl, cj = 16 * J + cl;
            for (int s4 = 0; s4 < n; s4 += 4) {
              const int row = s4 + g;
              const double u = (row < n && ci < m) ? Cm[ci * L.ldl + row] : 0.0;
              const double v = (row < n && cj < m) ? Cm[cj * L.ldl + row] : 0.0;
              acc = __builtin_amdgcn_mfma_f64_16x16x4f64(u, v, acc, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int R = 16 * I + g + 4 * r, Cc = 16 * J + cl;
              if (R < m && Cc < m && R >= Cc) Sm[Cc * L.ldm + R] = acc[r];
            }
          }
        wsync();
      }
#else
      // one entry (r, q), r >= q, per lane: independent dot products
      for (int e = lane; e < m * m; e += 64) {
        const int r = e % m, q = e / m;
        if (r >= q) Sm[q * L.ldm + r] = dot_strided(Cm + r * L.ldl, 1, Cm + q * L.ldl, n);
      }
#endif
#if SQR_S_REGS
      if (m <= 16) {
        // chol(S) with the rows of S in registers (lane i: row i), right-looking
        // as the register Cholesky of H above; the lower triangle back to Sm
        double sr[16], rdv = 1.0;
#pragma unroll
        for (int l = 0; l < 16; ++l) sr[l] = (lane < m && l <= lane) ? Sm[l * L.ldm + lane] : 0.0;
        bool bad = false;
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          if (j >= m) continue;  // wave-uniform
          const double d = bcast(sr[j], j);
          bad |= !(d > 0.0);
          const double ir = rsqrt_nr(d), r = d * ir;
          if (lane == j) {
            sr[j] = r;
            rdv = ir;
          } else if (lane > j) {
            sr[j] *= ir;
          }
#pragma unroll
          for (int l = j + 1; l < 16; ++l) sr[l] -= sr[j] * bcast(sr[j], l);
          __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int l = 0; l < 16; ++l)
          if (lane < m && l <= lane) Sm[l * L.ldm + lane] = sr[l];
        if (lane < m) lds[L.o_rdgs + lane] = rdv;
        wsync();
        if (bad) status = SQR_CHOL_S;
      } else
#endif
      if (!chol_lds(Sm, L.ldm, m, lds + L.o_rdgs, lane)) status = SQR_CHOL_S;
      SQ_STAMP(5);
    }
  }
  // ---- fused residuals: rd = A'y + G'z + c, rp = A x - b, the norms
  double r3[3] = {0.0, 0.0, 0.0};
  if (a.fuse_resid && status != SQR_DOMAIN) {
    // G'z: each column's eight row-lane partials (lanes 8j .. 8j+7)
    double d2 = 0.0;
#pragma unroll
    for (int q = 0; q < PEF; ++q) {
      double v = gz[q];
      v += row_partner<4>(v);
      v += row_partner<2>(v);
      v += row_partner<1>(v);
      const int col = (lane >> 3) + 8 * q;
      if ((lane & 7) == 0 && col < n) {
        double aty = 0.0;
        for (int r = 0; r < m; ++r) aty = fma(A[(int64_t)col * m + r], a.iy[p * m + r], aty);
        const double rd = (aty + v) + a.ic[p * n + col];
        a.odx[p * n + col] = -rd;
        d2 = fma(rd, rd, d2);
      }
    }
    double p2 = 0.0;
    if (lane < m) {
      double ax = 0.0;
      for (int j = 0; j < n; ++j) ax = fma(A[(int64_t)j * m + lane], a.ix[p * n + j], ax);
      const double rp = ax - a.ib[p * m + lane];
      a.ody[p * m + lane] = -rp;
      p2 = rp * rp;
    }
    r3[0] = sqrt(wave_sum(d2));
    r3[1] = sqrt(wave_sum(p2));
    r3[2] = wave_sum(zs);
  }
  // ---- the factor record
  if (status == 0) {
    // the lower triangle only: the record's upper triangle is zeroed once by
    // socp_sqr_create and never written
#pragma unroll
    for (int j = 0; j < NC; ++j)
      if (j < n && lane < n && lane >= j) rec[L.r_L + j * n + lane] = h[j];
    wsync();
    const double* Sm = lds + L.o_S;
    for (int e = lane; e < m * m; e += 64) {
      const int i = e % m, j = e / m;
      rec[L.r_S + e] = i >= j ? Sm[j * L.ldm + i] : 0.0;
    }
  }
  // the scaling whatever the factorisation did: compute_scaling runs (and
  // updates the SqrScaling object) before setup_iter's cholesky! can throw
  // (solver.jl:106,126)
  for (int i = lane; i < k; i += 64) {
    rec[L.r_l + i] = lds[L.o_l + i];
    rec[L.r_wb + i] = lds[L.o_wb + i];
  }
  for (int c = lane; c < nc; c += 64) rec[L.r_mu + c] = lds[L.o_mu + c];
  if (lane == 0) {
    rec[L.r_st] = (double)status;
    a.status[p] = status;
  }
  if (a.fuse_resid) {
    // socp_sqr_ipm_resid_kernel's decisions (solver.jl:106-125): the scaling's
    // DomainError first, then the exit test, then the factorisation's status
    int fin = -1;
    if (status == SQR_DOMAIN) {
      fin = SQR_DOMAIN;
    } else {
      if (lane == 0) {
        a.ores[3 * p + 0] = r3[0];
        a.ores[3 * p + 1] = r3[1];
        a.ores[3 * p + 2] = r3[2];
      }
      if (r3[0] + r3[1] + r3[2] < a.tol)
        fin = 0;
      else if (status != 0)
        fin = status;
    }
    if (fin >= 0) {
      if (lane == 0) {
        a.ostatus[p] = fin;
        a.oactive[p] = 0;
        atomicSub(a.n_active, 1);  // the host stops launching once none is left
      }
    } else {
      // ds = -(lam o lam) (vprod!, vectors.jl:58-81; the affine right-hand side)
      const double* lam = lds + L.o_l;
      for (int c = 0; c < nc; ++c) {
        const int o = a.cones.offs[c], d = a.cones.dim[c];
        if (a.cones.kind[c] == POC_K) {
          for (int i = o + lane; i < o + d; i += 64) a.ods[p * k + i] = -(lam[i] * lam[i]);
          continue;
        }
        double part = 0.0;
        for (int i = o + lane; i < o + d; i += 64) part += lam[i] * lam[i];
        const double t0 = wave_sum(part), l0 = lam[o];
        for (int i = o + 1 + lane; i < o + d; i += 64) a.ods[p * k + i] = -(l0 * lam[i] + l0 * lam[i]);
        if (lane == 0) a.ods[p * k + o] = -t0;
      }
    }
  }
  SQ_STAMP(6);
}

// -------------------------------------------------------- solve kernel
template <int NC>
__device__ __forceinline__ void solve_problem(Ctx& C, int64_t p) {
  const SqrArgs& a = C.a;
  const SqrLayout& L = C.L;
  double* lds = C.lds;
  const int lane = C.lane;
  const int n = a.n, m = a.m, k = a.k, nc = a.nc;
  const double* G = a.G + p * (int64_t)k * n;
  const double* A = m ? a.A + p * (int64_t)m * n : nullptr;
  const bool sing = a.sing && a.sing[p];
  const double* rec = a.rec + p * L.rec;
  if (a.active && !a.active[p]) return;
  const int status = (int)rec[L.r_st];
  if (status != 0) {
    const double nan = __builtin_nan("");
    for (int i = lane; i < n; i += 64) a.cx[p * n + i] = nan;
    for (int i = lane; i < m; i += 64) a.cy[p * m + i] = nan;
    for (int i = lane; i < k; i += 64) {
      a.cz[p * k + i] = nan;
      a.cs[p * k + i] = nan;
    }
    if (lane == 0) a.status[p] = status;
    return;
  }
  double *Sm = lds + L.o_S, *rdgs = lds + L.o_rdgs;
  for (int e = lane; e < m * m; e += 64) {
    const int i = e % m, j = e / m;
    if (i > j) Sm[j * L.ldm + i] = rec[L.r_S + e];
    if (i == j) rdgs[i] = 1.0 / rec[L.r_S + e];
  }
#ifdef SOCP_DIAG
  uint64_t st_last = __builtin_amdgcn_s_memtime();
#endif
  double *lam = lds + L.o_l, *wb = lds + L.o_wb, *mu = lds + L.o_mu;
  double *dz = lds + L.o_s, *ds = lds + L.o_z;  // the setup's s, z slots
  double *k0 = lds + L.o_D, *k1 = lds + L.o_iW, *k2 = lds + L.o_u, *kt = lds + L.o_v;
  double *nv = lds + L.o_nv, *mv = lds + L.o_mv;
  for (int i = lane; i < k; i += 64) {
    lam[i] = rec[L.r_l + i];
    wb[i] = rec[L.r_wb + i];
    dz[i] = a.dz[p * k + i];
    ds[i] = a.ds[p * k + i];
  }
  for (int c = lane; c < nc; c += 64) mu[c] = rec[L.r_mu + c];
  wsync();
  // k0 = lam \ ds; k1 = W k0; k2 = dz - k1; k1 = W^-1 W^-1 k2   (spsolver.jl:90-96)
  for (int c = 0; c < nc; ++c) {
    const int o = a.cones.offs[c], d = a.cones.dim[c], kd = a.cones.kind[c];
    cone_iprod(lam, ds, k0, o, d, kd, lane);
    cone_scale(wb, mu[c], k0, k1, o, d, kd, false, lane);
    for (int i = o + lane; i < o + d; i += 64) k2[i] = dz[i] - k1[i];
    cone_scale(wb, mu[c], k2, k1, o, d, kd, true, lane);
    cone_scale(wb, mu[c], k1, k1, o, d, kd, true, lane);
  }
  SQ_STAMP(8);
  // n0 = G' k1 + dx (+ A' dy)   (:97-102): a lane per column
  double n0 = 0.0;
  if (lane < n) {
    n0 = dot_strided<SQR_GU>(G + (int64_t)lane * k, 1, k1, k);
    n0 += a.dx[p * n + lane];
    if (sing) n0 += dot_strided(A + (int64_t)lane * m, 1, a.dy + p * m, m);
  }
  // the factor rows into registers (after the G' mat-vec: not live during it);
  // rows n..NC-1 as identity rows ([L 0; 0 I]): no guards in the solves
  double h[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) h[j] = (j < n && lane < n) ? rec[L.r_L + j * n + lane] : (lane == j ? 1.0 : 0.0);
  const double rd = lane < n ? 1.0 / rec[L.r_L + lane * n + lane] : 1.0;
  SQ_STAMP(9);
  // n1 = H^-1 n0 (:104-107)
  const double y0 = fwd_solve<NC>(h, rd, n, n0, lane);
  SQ_STAMP(10);
  const double n1 = bwd_solve<NC>(h, rd, n, y0, lane);
  SQ_STAMP(11);
  if (m > 0) {
    // m0 = A n1 - dy; cy = S^-1 m0; m0 = sing ? dy - cy : -cy   (:108-118)
    if (lane < n) nv[lane] = n1;
    wsync();
    double t = 0.0;
    if (lane < m) t = dot_strided(A + lane, m, nv, n) - a.dy[p * m + lane];
    const double cy = chol_solve_lds(Sm, L.ldm, rdgs, m, t, lane);
    if (lane < m) {
      a.cy[p * m + lane] = cy;
      const double dy = a.dy[p * m + lane];
      mv[lane] = (sing && !a.init) ? dy - cy : -cy;  // init: the exact KKT solution (solver.jl:84)
    }
    wsync();
    // n0 += A' m0   (:119-120)
    if (lane < n) n0 += dot_strided(A + (int64_t)lane * m, 1, mv, m);
  }
  SQ_STAMP(12);
  // cx = H^-1 n0 (:122-124)
  const double cx = bwd_solve<NC>(h, rd, n, fwd_solve<NC>(h, rd, n, n0, lane), lane);
  SQ_STAMP(13);
  if (lane < n) {
    a.cx[p * n + lane] = cx;
    nv[lane] = cx;
  }
  wsync();
  // k1 = G cx - k2 (:125-126), a lane per row
  for (int i = lane; i < k; i += 64) kt[i] = dot_strided<SQR_GU>(G + i, k, nv, n) - k2[i];
  // cz = W^-1 W^-1 k1; k1 = W cz; k0 -= k1; cs = W k0   (:127-131)
  double *cz = k2, *cs = k1;
  for (int c = 0; c < nc; ++c) {
    const int o = a.cones.offs[c], d = a.cones.dim[c], kd = a.cones.kind[c];
    cone_scale(wb, mu[c], kt, cz, o, d, kd, true, lane);
    cone_scale(wb, mu[c], cz, cz, o, d, kd, true, lane);
    cone_scale(wb, mu[c], cz, kt, o, d, kd, false, lane);
    for (int i = o + lane; i < o + d; i += 64) k0[i] -= kt[i];
    cone_scale(wb, mu[c], k0, cs, o, d, kd, false, lane);
  }
  wsync();
  for (int i = lane; i < k; i += 64) {
    a.cz[p * k + i] = cz[i];
    a.cs[p * k + i] = cs[i];
  }
  if (lane == 0) a.status[p] = 0;
  SQ_STAMP(14);
}


// ================================================ workgroup kernels (n, m <= 160)
// One SQR_LT-thread workgroup (4 wavefronts) per problem for shapes whose
// factor does not fit one wavefront's registers -- the reference's own
// optimal-control problem (runtests.jl:204-244, n = 150, m = 102) among them.
// The factor lives packed (lower triangle, column-major) in LDS; C = L^-1 A'
// is formed 16 right-hand sides at a time and kept in the record's scratch;
// H and S = C'C are lower 16 x 16 tiles of f64 MFMA 16x16x4 dealt out to the
// four wavefronts.  The cone operations run on wavefront 0 (the wavefront
// helpers above); the column recurrences take one barrier per column.

__device__ __forceinline__ void bar() { __syncthreads(); }

// lower 16x16 tiles of X'Y (+ X2'X2) into the packed LDS triangle P (N x N):
// X[r][a] = fa[r] * src[a * ld + r], Y[r][b] = fb[r] * src[b * ld + r] for
// r < rows (fa / fb NULL: 1); with src2, the unscaled rows of src2 (rows2 x N,
// leading dimension ld2) are added to the same accumulators.
__device__ __forceinline__ void syrk_tiles(const double* src, int ld, int rows, const double* fa, const double* fb,
                                           const double* src2, int ld2, int rows2, int N, double* P, int tid) {
  typedef double d4v __attribute__((ext_vector_type(4)));
  const int w = tid >> 6, lane = tid & 63, cl = lane & 15, kk = lane >> 4;
  const int NT = (N + 15) / 16;
  for (int t = w; t < NT * (NT + 1) / 2; t += SQR_LT / 64) {
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    const int J = t - I * (I + 1) / 2;
    const int a = 16 * I + cl, b = 16 * J + cl;
    const bool va = a < N, vb = b < N;
    d4v acc = {0.0, 0.0, 0.0, 0.0};
    for (int r0 = 0; r0 < rows; r0 += 4) {
      const int r = r0 + kk;
      const bool vr = r < rows;
      double xa = (vr && va) ? src[(int64_t)a * ld + r] : 0.0;
      double yb = (vr && vb) ? src[(int64_t)b * ld + r] : 0.0;
      if (fa && vr) xa *= fa[r];
      if (fb && vr) yb *= fb[r];
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(xa, yb, acc, 0, 0, 0);
    }
    if (src2)
      for (int r0 = 0; r0 < rows2; r0 += 4) {
        const int r = r0 + kk;
        const bool vr = r < rows2;
        const double xa = (vr && va) ? src2[(int64_t)a * ld2 + r] : 0.0;
        const double yb = (vr && vb) ? src2[(int64_t)b * ld2 + r] : 0.0;
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(xa, yb, acc, 0, 0, 0);
      }
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int row = 16 * I + kk + 4 * v, col = 16 * J + cl;
      if (row < N && col <= row) P[sqr_pk(row, col, N)] = acc[v];
    }
  }
}

// right-looking Cholesky of the packed N x N triangle; 1/diag -> rdg; false at
// a pivot <= 0 or NaN (the same value in every thread: a uniform exit)
__device__ __forceinline__ bool chol_packed(double* P, int N, double* rdg, int tid) {
  for (int j = 0; j < N; ++j) {
    bar();
    const double d = P[sqr_pk(j, j, N)];
    if (!(d > 0.0)) return false;
    const double ir = rsqrt_nr(d);
    bar();
    for (int i = j + tid; i < N; i += SQR_LT) {
      if (i == j) {
        P[sqr_pk(j, j, N)] = d * ir;
        rdg[j] = ir;
      } else {
        P[sqr_pk(i, j, N)] *= ir;
      }
    }
    bar();
    // trailing update L(i, l) -= L(i, j) L(l, j), j < l <= i: 16 x 16 thread grid
    const int ti = tid >> 4, tl = tid & 15;
    for (int l = j + 1 + tl; l < N; l += 16) {
      const double llj = P[sqr_pk(l, j, N)];
      for (int i = l + ti; i < N; i += 16) P[sqr_pk(i, l, N)] -= P[sqr_pk(i, j, N)] * llj;
    }
  }
  bar();
  return true;
}

// L y = b then L' x = y against the packed factor, b in LDS (N), in place
__device__ __forceinline__ void chol_solve_packed(const double* P, int N, const double* rdg, double* b, int tid) {
  for (int j = 0; j < N; ++j) {
    bar();
    const double xj = b[j] * rdg[j];
    bar();
    if (tid == 0) b[j] = xj;
    for (int i = j + 1 + tid; i < N; i += SQR_LT) b[i] -= P[sqr_pk(i, j, N)] * xj;
  }
  for (int j = N - 1; j >= 0; --j) {
    bar();
    const double xj = b[j] * rdg[j];
    bar();
    if (tid == 0) b[j] = xj;
    for (int i = tid; i < j; i += SQR_LT) b[i] -= P[sqr_pk(j, i, N)] * xj;
  }
  bar();
}

// the same two triangular solves against a column-major factor in global memory
// (the record's L_S: m x m, zeros above the diagonal)
__device__ __forceinline__ void chol_solve_global(const double* F, int N, double* b, int tid) {
  for (int j = 0; j < N; ++j) {
    bar();
    const double xj = b[j] / F[(int64_t)j * N + j];
    bar();
    if (tid == 0) b[j] = xj;
    for (int i = j + 1 + tid; i < N; i += SQR_LT) b[i] -= F[(int64_t)j * N + i] * xj;
  }
  for (int j = N - 1; j >= 0; --j) {
    bar();
    const double xj = b[j] / F[(int64_t)j * N + j];
    bar();
    if (tid == 0) b[j] = xj;
    for (int i = tid; i < j; i += SQR_LT) b[i] -= F[(int64_t)i * N + j] * xj;
  }
  bar();
}

__device__ __forceinline__ void setup_problem_wg(Ctx& C, int64_t p, int tid) {
  const SqrArgs& a = C.a;
  const SqrLayout& L = C.L;
  double* lds = C.lds;
  const int n = a.n, m = a.m, k = a.k, nc = a.nc;
  const double* G = a.G + p * (int64_t)k * n;
  const double* A = m ? a.A + p * (int64_t)m * n : nullptr;
  const bool sing = a.sing && a.sing[p];
  double* rec = a.rec + p * L.rec;
  if (a.active && !a.active[p]) return;  // uniform over the workgroup
  double* P = L.gfac ? rec + L.r_P : lds + L.o_L;  // the packed factor of H
  double* rdg = lds + L.o_nv;  // 1 / diag of the current factor
  for (int i = tid; i < k; i += SQR_LT) {
    lds[L.o_s + i] = a.s[p * k + i];
    lds[L.o_z + i] = a.z[p * k + i];
    lds[L.o_one + i] = 1.0;
  }
  if (tid == 0) lds[L.o_flag] = 0.0;
  bar();
  if (tid < 64)
    for (int c = 0; c < nc; ++c) sqr_scaling_cone(C, c);
  bar();
  int status = (int)lds[L.o_flag];
  if (status == 0) {
    // H = (iW G)'(iW G) (spsolver.jl:62-64), or G'(iWiW G) + A'A when sing (:67-71)
    if (!sing)
      syrk_tiles(G, k, k, lds + L.o_iW, lds + L.o_iW, nullptr, 0, 0, n, P, tid);
    else
      syrk_tiles(G, k, k, nullptr, lds + L.o_D, m ? A : nullptr, m, m, n, P, tid);
    if (!chol_packed(P, n, rdg, tid)) status = SQR_CHOL_H;
  }
  // modify_factors! (sqrscalings.jl:160-194): per SOC cone the update with
  // G'u and the downdate with G'v, the downdate chain one column behind
  for (int c = 0; c < nc && status == 0; ++c) {
    if (a.cones.kind[c] != SOC_K) continue;
    const int o = a.cones.offs[c], d = a.cones.dim[c];
    double *wu = lds + L.o_w, *wv = lds + L.o_wv;
    bar();
    for (int col = tid; col < n; col += SQR_LT) {
      double su = 0.0, sv = 0.0;
      for (int r = o; r < o + d; ++r) {
        const double g = G[(int64_t)col * k + r];
        su += g * lds[L.o_u + r];
        sv += g * lds[L.o_v + r];
      }
      wu[col] = su;
      wv[col] = sv;
    }
    bool bad = false;
    for (int t = 0; t <= n; ++t) {
      bar();
      // chain u at column t, chain v at column t - 1 (its column t - 1 is final for u)
      const int ju = t, jv = t - 1;
      double cu = 0, su_ = 0, iu = 0, cv = 0, sv_ = 0, iv = 0, ru = 0, rv = 0;
      if (ju < n) {
        const double ljj = P[sqr_pk(ju, ju, n)], wj = wu[ju];
        const double r2 = ljj * ljj + wj * wj;
        bad |= !(r2 > 0.0);
        const double ir = rsqrt_nr(r2);
        ru = r2 * ir;
        const double il = 1.0 / ljj;
        cu = ru * il;
        su_ = wj * il;
        iu = ljj * ir;
      }
      if (jv >= 0) {
        const double ljj = P[sqr_pk(jv, jv, n)], wj = wv[jv];
        const double r2 = ljj * ljj - wj * wj;
        bad |= !(r2 > 0.0);
        const double ir = rsqrt_nr(r2);
        rv = r2 * ir;
        const double il = 1.0 / ljj;
        cv = rv * il;
        sv_ = wj * il;
        iv = ljj * ir;
      }
      bar();
      if (ju < n) {
        for (int i = ju + 1 + tid; i < n; i += SQR_LT) {
          const double lij = (P[sqr_pk(i, ju, n)] + su_ * wu[i]) * iu;
          P[sqr_pk(i, ju, n)] = lij;
          wu[i] = cu * wu[i] - su_ * lij;
        }
        if (tid == 0) P[sqr_pk(ju, ju, n)] = ru;
      }
      if (jv >= 0) {
        for (int i = jv + 1 + tid; i < n; i += SQR_LT) {
          const double lij = (P[sqr_pk(i, jv, n)] - sv_ * wv[i]) * iv;
          P[sqr_pk(i, jv, n)] = lij;
          wv[i] = cv * wv[i] - sv_ * lij;
        }
        if (tid == 0) P[sqr_pk(jv, jv, n)] = rv;
      }
    }
    if (bad) status = SQR_CHOL_H;  // uniform: every thread evaluated the same pivots
  }
  bar();
  if (status == 0) {
    for (int j = tid; j < n; j += SQR_LT) rdg[j] = 1.0 / P[sqr_pk(j, j, n)];
    // the factor into the record (column-major, zeros above the diagonal)
    for (int e = tid; e < n * n; e += SQR_LT) {  // lower triangle (the upper one stays zero)
      const int i = e % n, j = e / n;
      if (i >= j) rec[L.r_L + e] = P[sqr_pk(i, j, n)];
    }
    bar();
    if (m > 0) {
      // C = L^-1 A' (spsolver.jl:80-82), SQR_RC right-hand sides at a time
      double* Cg = rec + L.r_C;   // C[q * n + i]
      for (int q0 = 0; q0 < m; q0 += SQR_RC) {
        const int nr = (m - q0) < SQR_RC ? (m - q0) : SQR_RC;
        double* Cc = L.gfac ? Cg + (int64_t)q0 * n : lds + L.o_C;  // Cc[t * n + i]
        bar();
        for (int e = tid; e < nr * n; e += SQR_LT) {
          const int t = e / n, i = e % n;
          Cc[t * n + i] = A[(int64_t)i * m + q0 + t];
        }
        for (int j = 0; j < n; ++j) {
          bar();
          const int t = tid & 15;
          const double xj = t < nr ? Cc[t * n + j] * rdg[j] : 0.0;
          bar();
          if (t < nr) {
            if ((tid >> 4) == 0) Cc[t * n + j] = xj;
            for (int i = j + 1 + (tid >> 4); i < n; i += SQR_LT / 16) Cc[t * n + i] -= P[sqr_pk(i, j, n)] * xj;
          }
        }
        bar();
        if (!L.gfac)
          for (int e = tid; e < nr * n; e += SQR_LT) Cg[(int64_t)q0 * n + e] = Cc[e];
      }
      __threadfence_block();
      bar();
      // S = C'C (:83) into the packed triangle (L_H is in the record now; with
      // gfac, S's own region: the solves read L_H packed), chol(S)
      double* PS = L.gfac ? rec + L.r_PS : P;
      syrk_tiles(Cg, n, n, nullptr, nullptr, nullptr, 0, 0, m, PS, tid);
      double* rds = lds + L.o_rdgs;
      if (!chol_packed(PS, m, rds, tid)) status = SQR_CHOL_S;
      if (status == 0)
        for (int e = tid; e < m * m; e += SQR_LT) {
          const int i = e % m, j = e / m;
          rec[L.r_S + e] = i >= j ? PS[sqr_pk(i, j, m)] : 0.0;
        }
    }
  }
  // the scaling whatever the factorisation did (compute_scaling precedes
  // setup_iter's cholesky!, solver.jl:106,126)
  for (int i = tid; i < k; i += SQR_LT) {
    rec[L.r_l + i] = lds[L.o_l + i];
    rec[L.r_wb + i] = lds[L.o_wb + i];
  }
  for (int c = tid; c < nc; c += SQR_LT) rec[L.r_mu + c] = lds[L.o_mu + c];
  if (tid == 0) {
    rec[L.r_st] = (double)status;
    a.status[p] = status;
  }
}

__device__ __forceinline__ void solve_problem_wg(Ctx& C, int64_t p, int tid) {
  const SqrArgs& a = C.a;
  const SqrLayout& L = C.L;
  double* lds = C.lds;
  const int n = a.n, m = a.m, k = a.k, nc = a.nc;
  const double* G = a.G + p * (int64_t)k * n;
  const double* A = m ? a.A + p * (int64_t)m * n : nullptr;
  const bool sing = a.sing && a.sing[p];
  const double* rec = a.rec + p * L.rec;
  if (a.active && !a.active[p]) return;  // uniform over the workgroup
  const int status = (int)rec[L.r_st];
  if (status != 0) {
    const double nan = __builtin_nan("");
    for (int i = tid; i < n; i += SQR_LT) a.cx[p * n + i] = nan;
    for (int i = tid; i < m; i += SQR_LT) a.cy[p * m + i] = nan;
    for (int i = tid; i < k; i += SQR_LT) {
      a.cz[p * k + i] = nan;
      a.cs[p * k + i] = nan;
    }
    if (tid == 0) a.status[p] = status;
    return;
  }
  double *lam = lds + L.o_l, *wb = lds + L.o_wb, *mu = lds + L.o_mu;
  double *dz = lds + L.o_s, *ds = lds + L.o_z;
  double *k0 = lds + L.o_D, *k1 = lds + L.o_iW, *k2 = lds + L.o_u, *kt = lds + L.o_v;
  double *n0 = lds + L.o_n0, *nb = lds + L.o_n1, *mv = lds + L.o_mv, *rdg = lds + L.o_nv;
  const double* P = L.gfac ? rec + L.r_P : lds + L.o_L;  // the packed factor of H
  for (int i = tid; i < k; i += SQR_LT) {
    lam[i] = rec[L.r_l + i];
    wb[i] = rec[L.r_wb + i];
    dz[i] = a.dz[p * k + i];
    ds[i] = a.ds[p * k + i];
  }
  for (int c = tid; c < nc; c += SQR_LT) mu[c] = rec[L.r_mu + c];
  if (!L.gfac)  // (with gfac the setup left it packed in the record)
    for (int e = tid; e < n * n; e += SQR_LT) {
      const int i = e % n, j = e / n;
      if (i >= j) lds[L.o_L + sqr_pk(i, j, n)] = rec[L.r_L + e];
    }
  for (int j = tid; j < n; j += SQR_LT) rdg[j] = 1.0 / rec[L.r_L + (int64_t)j * n + j];
  bar();
  // k0 = lam \\ ds; k1 = W k0; k2 = dz - k1; k1 = W^-1 W^-1 k2   (spsolver.jl:90-96)
  if (tid < 64)
    for (int c = 0; c < nc; ++c) {
      const int o = a.cones.offs[c], d = a.cones.dim[c], kd = a.cones.kind[c];
      cone_iprod(lam, ds, k0, o, d, kd, tid);
      cone_scale(wb, mu[c], k0, k1, o, d, kd, false, tid);
      for (int i = o + tid; i < o + d; i += 64) k2[i] = dz[i] - k1[i];
      cone_scale(wb, mu[c], k2, k1, o, d, kd, true, tid);
      cone_scale(wb, mu[c], k1, k1, o, d, kd, true, tid);
    }
  bar();
  // n0 = G' k1 + dx (+ A' dy)   (:97-102): a thread per column
  for (int col = tid; col < n; col += SQR_LT) {
    double v = dot_strided(G + (int64_t)col * k, 1, k1, k) + a.dx[p * n + col];
    if (sing) v += dot_strided(A + (int64_t)col * m, 1, a.dy + p * m, m);
    n0[col] = v;
    nb[col] = v;
  }
  // n1 = H^-1 n0 (:104-107)
  chol_solve_packed(P, n, rdg, nb, tid);
  if (m > 0) {
    // m0 = A n1 - dy; cy = S^-1 m0; m0 = sing ? dy - cy : -cy   (:108-118)
    for (int r = tid; r < m; r += SQR_LT) mv[r] = dot_strided(A + r, m, nb, n) - a.dy[p * m + r];
    chol_solve_global(rec + L.r_S, m, mv, tid);
    for (int r = tid; r < m; r += SQR_LT) {
      const double cy = mv[r], dy = a.dy[p * m + r];
      a.cy[p * m + r] = cy;
      mv[r] = (sing && !a.init) ? dy - cy : -cy;  // init: the exact KKT solution (solver.jl:84)
    }
    bar();
    // n0 += A' m0   (:119-120)
    for (int col = tid; col < n; col += SQR_LT) n0[col] += dot_strided(A + (int64_t)col * m, 1, mv, m);
  }
  // cx = H^-1 n0 (:122-124)
  chol_solve_packed(P, n, rdg, n0, tid);
  for (int col = tid; col < n; col += SQR_LT) a.cx[p * n + col] = n0[col];
  // k1 = G cx - k2 (:125-126), a thread per row
  for (int i = tid; i < k; i += SQR_LT) kt[i] = dot_strided(G + i, k, n0, n) - k2[i];
  bar();
  // cz = W^-1 W^-1 k1; k1 = W cz; k0 -= k1; cs = W k0   (:127-131)
  double *cz = k2, *cs = k1;
  if (tid < 64)
    for (int c = 0; c < nc; ++c) {
      const int o = a.cones.offs[c], d = a.cones.dim[c], kd = a.cones.kind[c];
      cone_scale(wb, mu[c], kt, cz, o, d, kd, true, tid);
      cone_scale(wb, mu[c], cz, cz, o, d, kd, true, tid);
      cone_scale(wb, mu[c], cz, kt, o, d, kd, false, tid);
      for (int i = o + tid; i < o + d; i += 64) k0[i] -= kt[i];
      cone_scale(wb, mu[c], k0, cs, o, d, kd, false, tid);
    }
  bar();
  for (int i = tid; i < k; i += SQR_LT) {
    a.cz[p * k + i] = cz[i];
    a.cs[p * k + i] = cs[i];
  }
  if (tid == 0) a.status[p] = 0;
}

}  // namespace

// NC = 64: the LDS layout (~20 KB at the C2 shape) admits 8 workgroups per
// CU, i.e. 2 waves per SIMD, so the register budget is 256 (no spills)
template <int NC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NC >= 64 ? 2 : 3))) void socp_sqr_setup_kernel(SqrArgs a) {
  extern __shared__ double lds_dyn[];
  const SqrLayout L = sqr_layout(a.n, a.m, a.k, a.nc);
  Ctx C{a, L, lds_dyn, (int)threadIdx.x};
  setup_problem<NC>(C, (int64_t)blockIdx.x);
}

template <int NC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NC >= 64 ? SQR_SOLVE_WPE : 3))) void socp_sqr_solve_kernel(SqrArgs a) {
  extern __shared__ double lds_dyn[];
  const SqrLayout L = sqr_solve_layout(a.n, a.m, a.k, a.nc);
  Ctx C{a, L, lds_dyn, (int)threadIdx.x};
  solve_problem<NC>(C, (int64_t)blockIdx.x);
}

// socp_sqr_solve_socp's iteration after setup_iter (solver.jl:127-150) in one
// launch: solve_kkt (affine), step1, solve_kkt (combined), step2 for one
// problem per wavefront.  The same device code as the four launches it
// replaces, so the iterates are bitwise theirs; the second solve's passes over
// G and the factor record follow the first within microseconds (L2 / MALL
// instead of HBM), and three launches and their record reloads go.
__device__ __forceinline__ void global_rw_fence() {
  // this wavefront's global stores visible to its own later loads from other
  // lanes: workgroup scope (one CU's write-through L1; an agent-scope fence
  // would write back and invalidate the XCD's L2 per problem)
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}
template <int NC>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(NC >= 64 ? SQR_SOLVE_WPE : 3))) void
socp_sqr_ipm_solves_kernel(SqrArgs a, SqrIpmArgs ia, int it) {
  extern __shared__ double lds_dyn[];
  const int64_t p = blockIdx.x;
  if (!ia.active[p]) return;
  const int lane = (int)threadIdx.x;
  const SqrLayout L = sqr_solve_layout(a.n, a.m, a.k, a.nc);
  Ctx C{a, L, lds_dyn, lane};
  solve_problem<NC>(C, p);  // affine (solver.jl:127)
  global_rw_fence();
  wsync();
  if (!ipm_step1_problem(ia, p, lds_dyn, lane)) return;
  global_rw_fence();
  wsync();
  solve_problem<NC>(C, p);  // combined (:141)
  global_rw_fence();
  wsync();
  ipm_step2_problem(ia, p, it, lds_dyn, lane);
}

__global__ __launch_bounds__(SQR_LT) void socp_sqr_setup_wg_kernel(SqrArgs a) {
  extern __shared__ double lds_dyn[];
  const SqrLayout L = sqr_layout(a.n, a.m, a.k, a.nc);
  const int tid = (int)threadIdx.x;
  Ctx C{a, L, lds_dyn, tid & 63};
  setup_problem_wg(C, (int64_t)blockIdx.x, tid);
}

__global__ __launch_bounds__(SQR_LT) void socp_sqr_solve_wg_kernel(SqrArgs a) {
  extern __shared__ double lds_dyn[];
  const SqrLayout L = sqr_layout(a.n, a.m, a.k, a.nc);
  const int tid = (int)threadIdx.x;
  Ctx C{a, L, lds_dyn, tid & 63};
  solve_problem_wg(C, (int64_t)blockIdx.x, tid);
}

// NC = n rounded up to 16; the workgroup kernels above SQR_NMAX
const void* sqr_setup_kernel_ptr(int n, int m) {
  if (n > SQR_NMAX || m > SQR_NMAX) return (const void*)socp_sqr_setup_wg_kernel;
  if (n <= 16) return (const void*)socp_sqr_setup_kernel<16>;
  if (n <= 32) return (const void*)socp_sqr_setup_kernel<32>;
  if (n <= 48) return (const void*)socp_sqr_setup_kernel<48>;
  return (const void*)socp_sqr_setup_kernel<64>;
}
const void* sqr_ipm_solves_kernel_ptr(int n, int m) {
  if (n > SQR_NMAX || m > SQR_NMAX) return nullptr;
  if (n <= 16) return (const void*)socp_sqr_ipm_solves_kernel<16>;
  if (n <= 32) return (const void*)socp_sqr_ipm_solves_kernel<32>;
  if (n <= 48) return (const void*)socp_sqr_ipm_solves_kernel<48>;
  return (const void*)socp_sqr_ipm_solves_kernel<64>;
}
const void* sqr_solve_kernel_ptr(int n, int m) {
  if (n > SQR_NMAX || m > SQR_NMAX) return (const void*)socp_sqr_solve_wg_kernel;
  if (n <= 16) return (const void*)socp_sqr_solve_kernel<16>;
  if (n <= 32) return (const void*)socp_sqr_solve_kernel<32>;
  if (n <= 48) return (const void*)socp_sqr_solve_kernel<48>;
  return (const void*)socp_sqr_solve_kernel<64>;
}

}  // namespace socp
