// socp_sqr_step.hpp -- the rank-update IPM's cone-vector helpers and its two
// step phases (solver.jl:128-150), one wavefront per problem: shared by the
// step kernels (socp_sqr_ipm.hip) and the fused two-solve kernel
// (socp_sqr.hip, socp_sqr_ipm_solves_kernel).
#pragma once
#include <hip/hip_runtime.h>

#include "socp_sqr.hpp"

namespace socp {
namespace {

__device__ __forceinline__ double ws64(double v) { return cone_allreduce_rows<false>(v, 4); }
__device__ __forceinline__ double wm64(double v) { return cone_allreduce_rows<true>(v, 4); }
__device__ __forceinline__ void wsy() {
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");
  __builtin_amdgcn_wave_barrier();
}
// Julia's max / min: NaN if either argument is NaN
__device__ __forceinline__ double jmax(double a, double b) { return (isnan(a) || isnan(b)) ? NAN : (a > b ? a : b); }
__device__ __forceinline__ double jmin(double a, double b) { return (isnan(a) || isnan(b)) ? NAN : (a < b ? a : b); }

// vprod! (vectors.jl:58-81): t = u o v, one wavefront
__device__ void vprod_w(const ConeTable& C, double* t, const double* u, const double* v, int lane) {
  wsy();
  for (int c = 0; c < C.nc; ++c) {
    const int o = C.offs[c], d = C.dim[c];
    if (C.kind[c] == POC_K) {
      for (int i = o + lane; i < o + d; i += 64) t[i] = u[i] * v[i];
      continue;
    }
    double part = 0.0;
    for (int i = o + lane; i < o + d; i += 64) part += u[i] * v[i];
    const double t0 = ws64(part), iu = u[o], iv = v[o];
    for (int i = o + 1 + lane; i < o + d; i += 64) t[i] = iu * v[i] + iv * u[i];
    wsy();
    if (lane == 0) t[o] = t0;
  }
  wsy();
}

// scale! (inv = false) / iscale! (inv = true) (scalings.jl:112-173) of a whole k-vector
__device__ void scale_all(const ConeTable& C, const double* wb, const double* mu, const double* x, double* out,
                          bool inv, int lane) {
  wsy();
  for (int c = 0; c < C.nc; ++c) {
    const int o = C.offs[c], d = C.dim[c];
    if (C.kind[c] == POC_K) {
      for (int i = o + lane; i < o + d; i += 64) out[i] = inv ? recip(wb[i]) * x[i] : wb[i] * x[i];
      continue;
    }
    double part = 0.0;
    for (int i = o + 1 + lane; i < o + d; i += 64) part += wb[i] * x[i];
    const double del = ws64(part), x0 = x[o], w0 = wb[o];
    const double iw = recip(1.0 + w0);
    const double cst = inv ? (-x0 + del * iw) : (x0 + del * iw);
    const double f = inv ? recip(mu[c]) : mu[c];
    for (int i = o + 1 + lane; i < o + d; i += 64) out[i] = f * (x[i] + cst * wb[i]);
    wsy();
    if (lane == 0) out[o] = inv ? f * (w0 * x0 - del) : f * (w0 * x0 + del);
  }
  wsy();
}

// scmax (mats.jl:42-86): the largest "negative excursion" of x in lambda-scaled space
__device__ double scmax_w(const ConeTable& C, const double* li, const double* xi, int lane, bool& dom) {
  double mx = -INFINITY;
  for (int c = 0; c < C.nc; ++c) {
    const int o = C.offs[c], d = C.dim[c];
    double val;
    if (C.kind[c] == POC_K) {
      double v = -INFINITY;
      for (int i = o + lane; i < o + d; i += 64) {
        const double q = -xi[i] * recip(li[i]);
        if (q > v) v = q;
      }
      val = wm64(v);
    } else {
      double pl = 0.0, pr = 0.0;
      for (int i = o + 1 + lane; i < o + d; i += 64) {
        pl += li[i] * li[i];
        pr += li[i] * xi[i];
      }
      const double ai = li[o] * li[o] - ws64(pl);
      dom |= ai < 0.0;
      const double a = rsqrt_nr(ai);
      const double r1 = a * li[o] * xi[o] - a * ws64(pr);
      const double cst = (r1 + xi[o]) * recip(a * li[o] + 1.0);
      double r2 = 0.0;
      for (int i = o + 1 + lane; i < o + d; i += 64) {
        const double q = a * (xi[i] - cst * a * li[i]);
        r2 += q * q;
      }
      val = sqrt_nr(ws64(r2)) - a * r1;
    }
    if (val > mx) mx = val;
  }
  return mx;
}

// compute_step (mats.jl:30-40)
__device__ double compute_step_w(const ConeTable& C, const double* l, const double* ds, const double* dz, int lane,
                                 bool& dom) {
  const double t = jmax(jmax(scmax_w(C, l, ds, lane, dom), scmax_w(C, l, dz, lane, dom)), 0.0);
  return t < 1.0 ? 1.0 : (t == INFINITY ? 0.0 : jmin(1.0, recip(t)));  // min(1, 1/t), NaN kept
}

// make_e! (vectors.jl:7-24) entry i
__device__ __forceinline__ double e_of(const ConeTable& C, int i) {
  for (int c = 0; c < C.nc; ++c) {
    const int o = C.offs[c], d = C.dim[c];
    if (i >= o && i < o + d) return (C.kind[c] == POC_K || i == o) ? 1.0 : 0.0;
  }
  return 0.0;
}

// step1 (solver.jl:128-140) for problem p: kt3 = W rz, kt2 = W^-1 rs,
// compute_step, rho, sigma, mu and the corrector's right-hand side.  Returns
// false (and retires the problem) on scmax's DomainError.
__device__ __forceinline__ bool ipm_step1_problem(const SqrIpmArgs& a, int64_t p, double* lds, int lane) {
  const int n = a.n, m = a.m, k = a.k, nc = a.nc;
  const int KP = (k + 1) / 2 * 2;
  double *lam = lds, *wb = lds + KP, *kt2 = lds + 2 * KP, *kt3 = lds + 3 * KP, *kt1 = lds + 4 * KP,
         *rzv = lds + 5 * KP, *rsv = lds + 6 * KP, *mu = lds + 7 * KP;
  const double* rec = a.rec + p * a.rec_stride;
  for (int i = lane; i < k; i += 64) {
    lam[i] = rec[a.r_l + i];
    wb[i] = rec[a.r_wb + i];
    rzv[i] = a.rz[p * k + i];
    rsv[i] = a.rs[p * k + i];
  }
  for (int c = lane; c < nc; c += 64) mu[c] = rec[a.r_mu + c];
  scale_all(a.cones, wb, mu, rzv, kt3, false, lane);
  scale_all(a.cones, wb, mu, rsv, kt2, true, lane);
  bool dom = false;
  const double t = compute_step_w(a.cones, lam, kt3, kt2, lane, dom);
  if (__any(dom)) {  // Julia's sqrt of a negative number (scmax)
    if (lane == 0) {
      a.status[p] = SQR_DOMAIN;
      a.active[p] = 0;
      atomicSub(a.n_active, 1);  // the host stops launching once none is left
    }
    return false;
  }
  double pl = 0.0, pk = 0.0;
  for (int i = lane; i < k; i += 64) {
    pl += lam[i] * lam[i];
    pk += kt2[i] * kt3[i];
  }
  const double ll = ws64(pl), kk = ws64(pk);
  const double rho = 1.0 - t - t * t * kk / ll;
  const double cr = jmax(0.0, jmin(1.0, rho));
  double sig = 1.0;
  if (a.sigma_exp == 3) {
    sig = cr * cr * cr;  // Julia literal_pow
  } else {
    for (int q = 0; q < a.sigma_exp; ++q) sig *= cr;
  }
  const double muipm = ll / a.deg, scf = 1.0 - sig;
  vprod_w(a.cones, kt1, kt2, kt3, lane);
  for (int i = lane; i < k; i += 64) {
    const double e = e_of(a.cones, i);
    a.ds[p * k + i] += sig * muipm * e - kt1[i];
    a.dz[p * k + i] *= scf;
  }
  for (int j = lane; j < n; j += 64) a.dx[p * n + j] *= scf;
  for (int i = lane; i < m; i += 64) a.dy[p * m + i] *= scf;
  return true;
}

// step2 (solver.jl:143-150): step = 0.99 compute_step and the update.
// Returns false (and retires the problem) on scmax's DomainError.
__device__ __forceinline__ bool ipm_step2_problem(const SqrIpmArgs& a, int64_t p, int it, double* lds, int lane) {
  const int n = a.n, m = a.m, k = a.k, nc = a.nc;
  const int KP = (k + 1) / 2 * 2;
  double *lam = lds, *wb = lds + KP, *kt2 = lds + 2 * KP, *kt3 = lds + 3 * KP, *rzv = lds + 5 * KP,
         *rsv = lds + 6 * KP, *mu = lds + 7 * KP;
  const double* rec = a.rec + p * a.rec_stride;
  for (int i = lane; i < k; i += 64) {
    lam[i] = rec[a.r_l + i];
    wb[i] = rec[a.r_wb + i];
    rzv[i] = a.rz[p * k + i];
    rsv[i] = a.rs[p * k + i];
  }
  for (int c = lane; c < nc; c += 64) mu[c] = rec[a.r_mu + c];
  scale_all(a.cones, wb, mu, rzv, kt3, false, lane);
  scale_all(a.cones, wb, mu, rsv, kt2, true, lane);
  bool dom = false;
  const double t = compute_step_w(a.cones, lam, kt3, kt2, lane, dom);
  if (__any(dom)) {
    if (lane == 0) {
      a.status[p] = SQR_DOMAIN;
      a.active[p] = 0;
      atomicSub(a.n_active, 1);  // the host stops launching once none is left
    }
    return false;
  }
  const double stp = t * a.step;
  for (int j = lane; j < n; j += 64) a.x[p * n + j] += a.rx[p * n + j] * stp;
  for (int i = lane; i < m; i += 64) a.y[p * m + i] += a.ry[p * m + i] * stp;
  for (int i = lane; i < k; i += 64) {
    a.z[p * k + i] += rzv[i] * stp;
    a.s[p * k + i] += rsv[i] * stp;
  }
  if (lane == 0) a.iters[p] = it + 1;
  return true;
}
}  // namespace
}  // namespace socp
