// socp_sqr.hip — the rank-update KKT plugin on gfx950: the reference's
// SqrScaling + SparseSolver (sqrscalings.jl:8-194, spsolver.jl:1-130), i.e.
// W^-2 = D + u u' - v v' per SOC cone, H = G'DG (+A'A) factored as L L', one
// rank-1 update with G'u and one downdate with G'v per SOC cone
// (modify_factors!), S = (L^-1 A')'(L^-1 A') factored, and solve_kkt by
// triangular solves.  CHOLMOD (the reference's factoriser) is replaced by a
// dense LDS-resident factor: the batch's problems are small and dense.
//
// One 256-thread workgroup (4 wavefronts) per problem, n, m <= 64, k <= 256.
//   setup kernel: s, z -> scaling (one wavefront per cone), H in 4x4
//     register blocks from G row chunks staged through LDS, right-looking
//     Cholesky in LDS, the rank-1 modifications and the triangular solves on
//     wavefront 0 with one row per lane (pivot values by readlane), the
//     factor record (L_H, L_S, lambda, wb, mu, status) to HBM.
//   solve kernel: the record back into LDS, cone ops per wavefront, G'v / Gv
//     mat-vecs over all four wavefronts, the four H and two S triangular
//     solves on wavefront 0.
#include <hip/hip_runtime.h>

#include "socp_sqr.hpp"

namespace socp {

namespace {

__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

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

struct Ctx {
  const SqrArgs& a;
  const SqrLayout& L;
  double* lds;
  int tid, lane, wave;
};

// ------------------------------------------------------------- cone ops
// scale! (inv = false) / iscale! (inv = true) of one cone (scalings.jl:112-157)
// by one wavefront; op may alias x (every element is read before it is written).
__device__ void cone_scale(const double* wb, double mu, const double* x, double* op, int o, int d,
                           int kind, bool inv, int lane) {
  wsync();
  if (kind == POC_K) {
    for (int i = o + lane; i < o + d; i += 64) op[i] = inv ? 1.0 / wb[i] * x[i] : wb[i] * x[i];
    return;
  }
  double part = 0.0;
  for (int i = o + 1 + lane; i < o + d; i += 64) part += wb[i] * x[i];
  const double del = wave_sum(part);
  const double x0 = x[o], w0 = wb[o];
  if (inv) {
    const double cst = (-x0 + del / (1.0 + w0));
    const double im = 1.0 / mu;
    for (int i = o + 1 + lane; i < o + d; i += 64) op[i] = im * (x[i] + cst * wb[i]);
    if (lane == 0) op[o] = im * (w0 * x0 - del);
  } else {
    const double cst = (x0 + del / (1.0 + w0));
    for (int i = o + 1 + lane; i < o + d; i += 64) op[i] = mu * (x[i] + cst * wb[i]);
    if (lane == 0) op[o] = mu * (w0 * x0 + del);
  }
  wsync();
}

// iprod! (vectors.jl:99-125): t = lam^-1 o v of one cone, closed form of the O(d^2) loop
__device__ void cone_iprod(const double* lam, const double* v, double* t, int o, int d, int kind, int lane) {
  wsync();
  if (kind == POC_K) {
    for (int i = o + lane; i < o + d; i += 64) t[i] = v[i] / lam[i];
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
  for (int i = o + 1 + lane; i < o + d; i += 64)
    t[i] = -v0 * lam[i] / a + v[i] / l0 + lam[i] * lv / (l0 * a);
  if (lane == 0) t[o] = v0 * l0 / a - lv / a;
  wsync();
}

// ------------------------------------------------------------ scaling
// compute_scaling(::SqrScaling) (sqrscalings.jl:50-58, 66-139) of cone c
__device__ void sqr_scaling_cone(Ctx& C, int c) {
  const SqrLayout& L = C.L;
  double* lds = C.lds;
  const int kind = C.a.cones.kind[c], o = C.a.cones.offs[c], d = C.a.cones.dim[c];
  const double *s = lds + L.o_s, *z = lds + L.o_z;
  double *D = lds + L.o_D, *iW = lds + L.o_iW, *u = lds + L.o_u, *v = lds + L.o_v;
  double *lam = lds + L.o_l, *wb = lds + L.o_wb;
  bool bad = false;
  if (kind == POC_K) {
    for (int i = o + C.lane; i < o + d; i += 64) {
      const double zs = z[i] / s[i], sz = s[i] * z[i], sdz = s[i] / z[i];
      bad |= zs < 0.0 || sz < 0.0 || sdz < 0.0;
      D[i] = zs;
      iW[i] = sqrt(zs);
      lam[i] = sqrt(sz);
      wb[i] = sqrt(sdz);
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
    const double fs = 1.0 / sqrt(sprod), fz = 1.0 / sqrt(zprod);
    double pn = 0.0;
    for (int i = o + C.lane; i < o + d; i += 64) pn += (z[i] * fz) * (s[i] * fs);
    const double nsum = wave_sum(pn);
    bad |= (1.0 + nsum) < 0.0;
    const double gamma = sqrt((1.0 + nsum) / 2.0);
    const double s0 = s[o] * fs, z0 = z[o] * fz;
    const double wb0 = (s0 + z0) / (2.0 * gamma);
    double pw = 0.0;
    for (int i = o + 1 + C.lane; i < o + d; i += 64) {
      const double w = (s[i] * fs - z[i] * fz) / (2.0 * gamma);
      wb[i] = w;
      pw += w * w;
    }
    const double wb1sq = wave_sum(pw);
    const double q = sprod / zprod;
    bad |= q < 0.0;
    const double rq = sqrt(q);
    const double mu = sqrt(rq);
    const double inusq = 1.0 / rq, inu = 1.0 / mu;
    const double cv = -(1.0 + wb0 + wb1sq / (1.0 + wb0));
    const double dd = 1.0 + 2.0 / (1.0 + wb0) + wb1sq / ((1.0 + wb0) * (1.0 + wb0));
    const double av = (wb0 * wb0 + wb1sq - cv * cv * wb1sq / (1.0 + dd * wb1sq)) / 2.0;
    const double u0a = wb0 * wb0 + wb1sq - av;
    bad |= u0a < 0.0;
    const double u0 = sqrt(u0a);
    const double u1 = cv / u0;
    const double v1a = cv * cv / (u0 * u0) - dd;
    bad |= v1a < 0.0;
    const double v1 = sqrt(v1a);
    const double tmv1 = sqrt(sqrt(sprod) * sqrt(zprod));
    const double mult = tmv1 / (z0 + s0 + 2.0 * gamma);
    for (int i = o + 1 + C.lane; i < o + d; i += 64) {
      D[i] = inusq;
      iW[i] = sqrt(inusq);
      const double wbv = inu * wb[i];
      u[i] = u1 * wbv;
      v[i] = v1 * wbv;
      lam[i] = ((s[i] * fs) * (gamma + z0) + (z[i] * fz) * (gamma + s0)) * mult;
    }
    if (C.lane == 0) {
      D[o] = av * inusq;
      iW[o] = sqrt(fabs(av * inusq));
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

// ------------------------------------------------------------ Cholesky
// Right-looking L L' of the lower triangle of M (column-major, leading
// dimension ld, order n) by the whole workgroup.  The diagonal goes to dg[]
// (M's own diagonal entries are left stale).  Returns false at a pivot <= 0 or
// NaN (cholesky! throws PosDefException there).
__device__ bool chol_wg(Ctx& C, double* M, int ld, int n, double* dg) {
  for (int j = 0; j < n; ++j) {
    const double djj = M[j * ld + j];
    if (!(djj > 0.0)) return false;  // uniform: every thread read the same value
    const double r = sqrt(djj), ir = 1.0 / r;
    __syncthreads();
    if (C.tid == 0) dg[j] = r;
    for (int i = j + 1 + C.tid; i < n; i += 256) M[j * ld + i] *= ir;
    __syncthreads();
    const int i = C.lane;
    for (int l = j + 1 + C.wave; l < n; l += 4)
      if (i >= l && i < n) M[l * ld + i] -= M[j * ld + i] * M[j * ld + l];
    __syncthreads();
  }
  return true;
}

// forward (L y = b) then backward (L' x = y) solve by one wavefront, b one
// value per lane (rows), n <= 64
__device__ double chol_solve_wave(const double* M, int ld, const double* dg, int n, double b, int lane) {
  for (int j = 0; j < n; ++j) {
    const double xj = bcast(b, j) / dg[j];
    if (lane == j) b = xj;
    if (lane > j && lane < n) b -= M[j * ld + lane] * xj;
  }
  for (int j = n - 1; j >= 0; --j) {
    const double xj = bcast(b, j) / dg[j];
    if (lane == j) b = xj;
    if (lane < j) b -= M[lane * ld + j] * xj;
  }
  return b;
}

// -------------------------------------------------------- setup kernel
__device__ void setup_problem(Ctx& C, int64_t p) {
  const SqrArgs& a = C.a;
  const SqrLayout& L = C.L;
  double* lds = C.lds;
  const int n = a.n, m = a.m, k = a.k, nc = a.nc;
  const double* G = a.G + p * (int64_t)k * n;
  const double* A = m ? a.A + p * (int64_t)m * n : nullptr;
  const bool sing = a.sing && a.sing[p];
  double* rec = a.rec + p * L.rec;
  for (int i = C.tid; i < k; i += 256) {
    lds[L.o_s + i] = a.s[p * k + i];
    lds[L.o_z + i] = a.z[p * k + i];
  }
  if (C.tid == 0) lds[L.o_flag] = 0.0;
  __syncthreads();
  for (int c = C.wave; c < nc; c += 4) sqr_scaling_cone(C, c);
  __syncthreads();
  int status = (int)lds[L.o_flag];
  if (status == 0) {
    // ---- H = G'DG (+A'A): 4x4 blocks per thread, G row chunks via LDS
    double* M = lds + L.o_L;
    const int bi = C.tid >> 4, bj = C.tid & 15;
    const bool act = 4 * bi < n && 4 * bj < n;
    double acc[4][4];
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) acc[x][y] = 0.0;
    double *Ya = lds + L.o_X, *Yb = Ya + SQR_KC * SQR_NW;
    const double *fa = lds + (sing ? L.o_one : L.o_iW), *fb = lds + (sing ? L.o_D : L.o_iW);
    if (sing)
      for (int i = C.tid; i < k; i += 256) lds[L.o_one + i] = 1.0;
    for (int r0 = 0; r0 < k; r0 += SQR_KC) {
      __syncthreads();
      for (int e = C.tid; e < SQR_KC * 64; e += 256) {
        const int col = e / SQR_KC, r = e % SQR_KC;
        double g = 0.0, ga = 0.0, gb = 0.0;
        if (col < n && r0 + r < k) {
          g = G[(int64_t)col * k + r0 + r];
          ga = fa[r0 + r] * g;
          gb = fb[r0 + r] * g;
        }
        Ya[r * SQR_NW + col] = sing ? g : ga;
        Yb[r * SQR_NW + col] = gb;
      }
      __syncthreads();
      if (act) {
        const int rn = k - r0 < SQR_KC ? k - r0 : SQR_KC;
        for (int r = 0; r < rn; ++r) {
          double va[4], vb[4];
#pragma unroll
          for (int x = 0; x < 4; ++x) {
            va[x] = Ya[r * SQR_NW + 4 * bi + x];
            vb[x] = Yb[r * SQR_NW + 4 * bj + x];
          }
#pragma unroll
          for (int x = 0; x < 4; ++x)
#pragma unroll
            for (int y = 0; y < 4; ++y) acc[x][y] += va[x] * vb[y];
        }
      }
    }
    if (act) {
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const int i = 4 * bi + x, j = 4 * bj + y;
          if (i < n && j < n && i >= j) {
            double h = acc[x][y];
            if (sing) {
              double aa = 0.0;
              for (int r = 0; r < m; ++r) aa += A[(int64_t)i * m + r] * A[(int64_t)j * m + r];
              h += aa;
            }
            M[j * L.ldl + i] = h;
          }
        }
    }
    __syncthreads();
    double* dg = lds + L.o_dg;
    if (!chol_wg(C, M, L.ldl, n, dg)) status = SQR_CHOL_H;
    // ---- modify_factors! (sqrscalings.jl:160-194)
    for (int c = 0; c < nc && status == 0; ++c) {
      if (a.cones.kind[c] != SOC_K) continue;
      const int o = a.cones.offs[c], d = a.cones.dim[c];
      __syncthreads();
      if (C.tid < 128) {
        const int sel = C.tid >> 6, i = C.tid & 63;
        const double* uv = lds + (sel ? L.o_v : L.o_u);
        double w = 0.0;
        if (i < n)
          for (int r = o; r < o + d; ++r) w += G[(int64_t)i * k + r] * uv[r];
        lds[L.o_w + sel * 64 + i] = w;
      }
      __syncthreads();
      if (C.wave == 0) {
        bool ok = true;
        for (int sel = 0; sel < 2 && ok; ++sel) {
          const double sig = sel ? -1.0 : 1.0;
          double w = lds[L.o_w + sel * 64 + C.lane];
          for (int j = 0; j < n; ++j) {
            const double ljj = dg[j], wj = bcast(w, j);
            const double r2 = ljj * ljj + sig * wj * wj;
            if (!(r2 > 0.0)) {
              ok = false;
              break;
            }
            const double r = sqrt(r2);
            const double cc = r / ljj, sn = wj / ljj;
            if (C.lane == j) dg[j] = r;
            if (C.lane > j && C.lane < n) {
              const double lij = (M[j * L.ldl + C.lane] + sig * sn * w) / cc;
              M[j * L.ldl + C.lane] = lij;
              w = cc * w - sn * lij;
            }
          }
          wsync();
        }
        if (!ok && C.lane == 0) lds[L.o_flag] = (double)SQR_CHOL_H;
      }
      __syncthreads();
      status = (int)lds[L.o_flag];
    }
    // ---- C = L^-1 A' (m right-hand sides), S = C'C, chol(S)
    if (status == 0 && m > 0) {
      double* Cm = lds + L.o_X;  // the chunk buffers are free now
      __syncthreads();
      for (int q = C.wave; q < m; q += 4) {
        double b = C.lane < n ? A[(int64_t)C.lane * m + q] : 0.0;
        for (int j = 0; j < n; ++j) {
          const double xj = bcast(b, j) / dg[j];
          if (C.lane == j) b = xj;
          if (C.lane > j && C.lane < n) b -= M[j * L.ldl + C.lane] * xj;
        }
        if (C.lane < n) Cm[q * L.ldl + C.lane] = b;
      }
      __syncthreads();
      double* Sm = lds + L.o_S;
      for (int e = C.tid; e < m * m; e += 256) {
        const int r = e % m, q = e / m;
        if (r >= q) {
          double s = 0.0;
          for (int i = 0; i < n; ++i) s += Cm[r * L.ldl + i] * Cm[q * L.ldl + i];
          Sm[q * L.ldm + r] = s;
        }
      }
      __syncthreads();
      if (!chol_wg(C, Sm, L.ldm, m, lds + L.o_dgs)) status = SQR_CHOL_S;
    }
  }
  __syncthreads();
  // ---- the factor record
  if (status == 0) {
    const double* M = lds + L.o_L;
    for (int e = C.tid; e < n * n; e += 256) {
      const int i = e % n, j = e / n;
      rec[L.r_L + e] = i > j ? M[j * L.ldl + i] : (i == j ? lds[L.o_dg + j] : 0.0);
    }
    const double* Sm = lds + L.o_S;
    for (int e = C.tid; e < m * m; e += 256) {
      const int i = e % m, j = e / m;
      rec[L.r_S + e] = i > j ? Sm[j * L.ldm + i] : (i == j ? lds[L.o_dgs + j] : 0.0);
    }
    for (int i = C.tid; i < k; i += 256) {
      rec[L.r_l + i] = lds[L.o_l + i];
      rec[L.r_wb + i] = lds[L.o_wb + i];
    }
    for (int c = C.tid; c < nc; c += 256) rec[L.r_mu + c] = lds[L.o_mu + c];
  }
  if (C.tid == 0) {
    rec[L.r_st] = (double)status;
    a.status[p] = status;
  }
}

// -------------------------------------------------------- solve kernel
__device__ void solve_problem(Ctx& C, int64_t p) {
  const SqrArgs& a = C.a;
  const SqrLayout& L = C.L;
  double* lds = C.lds;
  const int n = a.n, m = a.m, k = a.k, nc = a.nc;
  const double* G = a.G + p * (int64_t)k * n;
  const double* A = m ? a.A + p * (int64_t)m * n : nullptr;
  const bool sing = a.sing && a.sing[p];
  const double* rec = a.rec + p * L.rec;
  const int status = (int)rec[L.r_st];
  if (status != 0) {
    const double nan = __builtin_nan("");
    for (int i = C.tid; i < n; i += 256) a.cx[p * n + i] = nan;
    for (int i = C.tid; i < m; i += 256) a.cy[p * m + i] = nan;
    for (int i = C.tid; i < k; i += 256) {
      a.cz[p * k + i] = nan;
      a.cs[p * k + i] = nan;
    }
    if (C.tid == 0) a.status[p] = status;
    return;
  }
  double *M = lds + L.o_L, *Sm = lds + L.o_S, *dg = lds + L.o_dg, *dgs = lds + L.o_dgs;
  for (int e = C.tid; e < n * n; e += 256) {
    const int i = e % n, j = e / n;
    if (i > j) M[j * L.ldl + i] = rec[L.r_L + e];
    if (i == j) dg[i] = rec[L.r_L + e];
  }
  for (int e = C.tid; e < m * m; e += 256) {
    const int i = e % m, j = e / m;
    if (i > j) Sm[j * L.ldm + i] = rec[L.r_S + e];
    if (i == j) dgs[i] = rec[L.r_S + e];
  }
  double *lam = lds + L.o_l, *wb = lds + L.o_wb, *mu = lds + L.o_mu;
  double *dz = lds + L.o_s, *ds = lds + L.o_z;  // the setup's s, z slots
  double *k0 = lds + L.o_D, *k1 = lds + L.o_iW, *k2 = lds + L.o_u, *kt = lds + L.o_v;
  double *nv = lds + L.o_w, *n1 = nv + 64, *mv = lds + L.o_mv;
  for (int i = C.tid; i < k; i += 256) {
    lam[i] = rec[L.r_l + i];
    wb[i] = rec[L.r_wb + i];
    dz[i] = a.dz[p * k + i];
    ds[i] = a.ds[p * k + i];
  }
  for (int c = C.tid; c < nc; c += 256) mu[c] = rec[L.r_mu + c];
  __syncthreads();
  // k0 = lam \ ds; k1 = W k0; k2 = dz - k1; k1 = W^-1 W^-1 k2   (spsolver.jl:90-96)
  for (int c = C.wave; c < nc; c += 4) {
    const int o = a.cones.offs[c], d = a.cones.dim[c], kd = a.cones.kind[c];
    cone_iprod(lam, ds, k0, o, d, kd, C.lane);
    cone_scale(wb, mu[c], k0, k1, o, d, kd, false, C.lane);
    wsync();
    for (int i = o + C.lane; i < o + d; i += 64) k2[i] = dz[i] - k1[i];
    cone_scale(wb, mu[c], k2, k1, o, d, kd, true, C.lane);
    cone_scale(wb, mu[c], k1, k1, o, d, kd, true, C.lane);
  }
  __syncthreads();
  // n0 = G' k1 + dx (+ A' dy)   (:97-102): one column per wavefront pass
  for (int col = C.wave; col < n; col += 4) {
    double part = 0.0;
    for (int i = C.lane; i < k; i += 64) part += G[(int64_t)col * k + i] * k1[i];
    double t = wave_sum(part) + a.dx[p * n + col];
    if (sing) {
      double s2 = 0.0;
      for (int r = C.lane; r < m; r += 64) s2 += A[(int64_t)col * m + r] * a.dy[p * m + r];
      t += wave_sum(s2);
    }
    if (C.lane == 0) nv[col] = t;
  }
  __syncthreads();
  // n1 = H^-1 n0 (:104-107)
  if (C.wave == 0) {
    const double b = chol_solve_wave(M, L.ldl, dg, n, C.lane < n ? nv[C.lane] : 0.0, C.lane);
    if (C.lane < n) n1[C.lane] = b;
  }
  __syncthreads();
  if (m > 0) {
    // m0 = A n1 - dy; cy = S^-1 m0; m0 = sing ? dy - cy : -cy   (:108-118)
    if (C.wave == 0) {
      double t = 0.0;
      if (C.lane < m) {
        for (int j = 0; j < n; ++j) t += A[(int64_t)j * m + C.lane] * n1[j];
        t -= a.dy[p * m + C.lane];
      }
      const double cy = chol_solve_wave(Sm, L.ldm, dgs, m, t, C.lane);
      if (C.lane < m) {
        a.cy[p * m + C.lane] = cy;
        const double dy = a.dy[p * m + C.lane];
        mv[C.lane] = sing ? dy - cy : -cy;
      }
    }
    __syncthreads();
    // n0 += A' m0   (:119-120)
    for (int j = C.tid; j < n; j += 256) {
      double t = 0.0;
      for (int r = 0; r < m; ++r) t += A[(int64_t)j * m + r] * mv[r];
      nv[j] += t;
    }
    __syncthreads();
  }
  // cx = H^-1 n0 (:122-124)
  if (C.wave == 0) {
    const double b = chol_solve_wave(M, L.ldl, dg, n, C.lane < n ? nv[C.lane] : 0.0, C.lane);
    if (C.lane < n) {
      n1[C.lane] = b;
      a.cx[p * n + C.lane] = b;
    }
  }
  __syncthreads();
  // k1 = G cx - k2 (:125-126), one row per thread
  for (int i = C.tid; i < k; i += 256) {
    double t = 0.0;
    for (int j = 0; j < n; ++j) t += G[(int64_t)j * k + i] * n1[j];
    kt[i] = t - k2[i];
  }
  __syncthreads();
  // cz = W^-1 W^-1 k1; k1 = W cz; k0 -= k1; cs = W k0   (:127-131)
  double *cz = k2, *cs = k1;
  for (int c = C.wave; c < nc; c += 4) {
    const int o = a.cones.offs[c], d = a.cones.dim[c], kd = a.cones.kind[c];
    cone_scale(wb, mu[c], kt, cz, o, d, kd, true, C.lane);
    cone_scale(wb, mu[c], cz, cz, o, d, kd, true, C.lane);
    cone_scale(wb, mu[c], cz, kt, o, d, kd, false, C.lane);
    wsync();
    for (int i = o + C.lane; i < o + d; i += 64) k0[i] -= kt[i];
    cone_scale(wb, mu[c], k0, cs, o, d, kd, false, C.lane);
  }
  __syncthreads();
  for (int i = C.tid; i < k; i += 256) {
    a.cz[p * k + i] = cz[i];
    a.cs[p * k + i] = cs[i];
  }
  if (C.tid == 0) a.status[p] = 0;
}

}  // namespace

__global__ __launch_bounds__(256) void socp_sqr_setup_kernel(SqrArgs a) {
  extern __shared__ double lds_dyn[];
  const SqrLayout L = sqr_layout(a.n, a.m, a.k, a.nc);
  Ctx C{a, L, lds_dyn, (int)threadIdx.x, (int)(threadIdx.x & 63), (int)(threadIdx.x >> 6)};
  setup_problem(C, (int64_t)blockIdx.x);
}

__global__ __launch_bounds__(256) void socp_sqr_solve_kernel(SqrArgs a) {
  extern __shared__ double lds_dyn[];
  const SqrLayout L = sqr_layout(a.n, a.m, a.k, a.nc);
  Ctx C{a, L, lds_dyn, (int)threadIdx.x, (int)(threadIdx.x & 63), (int)(threadIdx.x >> 6)};
  solve_problem(C, (int64_t)blockIdx.x);
}

const void* sqr_setup_kernel_ptr() { return (const void*)socp_sqr_setup_kernel; }
const void* sqr_solve_kernel_ptr() { return (const void*)socp_sqr_solve_kernel; }

}  // namespace socp
