// socp_sqr_ipm.hip — solve_socp (solver.jl:40-153) over a batch on the
// rank-update plugin: the reference's own tested configuration,
// SolverState(prob, SparseSolver(prob)) (runtests.jl:143-144, 188-189, 204-244),
// batched.  The host (socp_api.hip: socp_sqr_solve_socp) runs the iteration
// loop over the whole batch; each step below is one launch, one wavefront per
// problem, and problems that have stopped (converged, failed) are masked out
// of every launch, the factorisation and the KKT solves included.  Per
// iteration, in the reference's order:
//   setup   (socp_sqr.hip)  compute_scaling (sqrscalings.jl:50-139) + setup_iter (spsolver.jl:60-84)
//   resid   residuals and exit test (solver.jl:109-124), ds = lam o lam, RHS negation
//   solve   (socp_sqr.hip)  solve_kkt, affine (solver.jl:127)
//   step1   kt3 = W rz, kt2 = W^-1 rs, compute_step, rho, sigma, mu, corrector RHS (:128-140)
//   solve   (socp_sqr.hip)  solve_kkt, combined (:141)
//   step2   compute_step * 0.99 and the update (:143-150)
// The initial point (solver.jl:68-104) is the KKT system with W = I: setup
// at s = z = e, one solve with (-c, b, h, 0), then the cone shift.
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

// max_step (mats.jl:1-28)
__device__ double max_step_w(const ConeTable& C, const double* x, int lane) {
  double mx = -INFINITY;
  for (int c = 0; c < C.nc; ++c) {
    const int o = C.offs[c], d = C.dim[c];
    double val;
    if (C.kind[c] == POC_K) {
      double mn = INFINITY;
      for (int i = o + lane; i < o + d; i += 64) mn = x[i] < mn ? x[i] : mn;
      val = wm64(-mn);  // -min
    } else {
      double sq = 0.0;
      for (int i = o + 1 + lane; i < o + d; i += 64) sq += x[i] * x[i];
      val = sqrt_nr(ws64(sq)) - x[o];
    }
    if (val > mx) mx = val;
  }
  return mx;
}

// make_e! (vectors.jl:7-24) entry i
__device__ __forceinline__ double e_of(const ConeTable& C, int i) {
  for (int c = 0; c < C.nc; ++c) {
    const int o = C.offs[c], d = C.dim[c];
    if (i >= o && i < o + d) return (C.kind[c] == POC_K || i == o) ? 1.0 : 0.0;
  }
  return 0.0;
}

// rd = A'y + G'z + c (into rdv, n), rp = Ax - b (m), rz = Gx + s - h (k); returns
// (||rd||, ||rp||, z's) -- solver.jl:109-118, 122.
// One pass over the columns of G and A (column-major: a column is contiguous,
// so a lane per row reads coalesced), 16 columns at a time: every lane keeps
// its rows' G x and A x running sums, and its share of the column dot
// products G'z + A'y, which a reduce-scatter over the 16 lanes of a row and a
// sum over the four rows turn into the 16 columns' totals (lane cl of every
// row holds column j0 + cl).  k, m <= 256: four rows per lane (beyond, a
// two-pass form).
__device__ void residuals_w(const SqrIpmArgs& a, int64_t p, double* rdv, double* rpv, double* rzv, double (&r3)[3],
                            int lane) {
  const int n = a.n, m = a.m, k = a.k;
  const double* G = a.G + p * (int64_t)k * n;
  const double* A = m ? a.A + p * (int64_t)m * n : nullptr;
  const double *x = a.x + p * n, *y = a.y + p * m, *z = a.z + p * k, *s = a.s + p * k;
  const int cl = lane & 15;
  if (k > 256 || m > 256) {
    // beyond four rows per lane (the workgroup plugin's large shapes): the
    // column dot products a column at a time (a wave sum each), then the row
    // sums a lane per row -- the same sums, summed in another order
    double d2 = 0.0, p2 = 0.0, zs = 0.0;
    for (int j = 0; j < n; ++j) {
      const double* Gj = G + (int64_t)j * k;
      double pc = 0.0;
      for (int i = lane; i < k; i += 64) pc = fma(Gj[i], z[i], pc);
      if (m) {
        const double* Aj = A + (int64_t)j * m;
        for (int i = lane; i < m; i += 64) pc = fma(Aj[i], y[i], pc);
      }
      const double v = ws64(pc) + a.c[p * n + j];
      if (lane == 0) rdv[j] = v;
      d2 += v * v;  // every lane holds v: d2 is the same in all lanes
    }
    for (int i = lane; i < k; i += 64) {
      double gx = 0.0;
      for (int j = 0; j < n; ++j) gx = fma(G[(int64_t)j * k + i], x[j], gx);
      if (rzv) rzv[i] = gx + s[i] - a.h[p * k + i];
      zs += z[i] * s[i];
    }
    for (int i = lane; i < m; i += 64) {
      double ax = 0.0;
      for (int j = 0; j < n; ++j) ax = fma(A[(int64_t)j * m + i], x[j], ax);
      const double v = ax - a.b[p * m + i];
      rpv[i] = v;
      p2 += v * v;
    }
    r3[0] = sqrt(d2);
    r3[1] = sqrt(ws64(p2));
    r3[2] = ws64(zs);
    return;
  }
  constexpr int R = 4;
  double zr[R], yr[R], gx[R], ax[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int i = lane + 64 * r;
    zr[r] = i < k ? z[i] : 0.0;
    yr[r] = i < m ? y[i] : 0.0;
    gx[r] = 0.0;
    ax[r] = 0.0;
  }
  double d2 = 0.0, p2 = 0.0, zs = 0.0;
  for (int j0 = 0; j0 < n; j0 += 16) {
    double P[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const int j = j0 + c;
      double pc = 0.0;
      if (j < n) {  // wave-uniform
        const double xj = x[j];
        const double* Gj = G + (int64_t)j * k;
        const double* Aj = m ? A + (int64_t)j * m : nullptr;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int i = lane + 64 * r;
          if (64 * r < k) {  // wave-uniform
            const double gv = i < k ? Gj[i] : 0.0;
            pc = fma(gv, zr[r], pc);
            gx[r] = fma(gv, xj, gx[r]);
          }
          if (64 * r < m) {
            const double av = i < m ? Aj[i] : 0.0;
            pc = fma(av, yr[r], pc);
            ax[r] = fma(av, xj, ax[r]);
          }
        }
      }
      P[c] = pc;
    }
    int base = 0;
    rs16<16, 8>(P, cl, base);  // base == cl: this row's partial of column j0 + cl
    const double tot = rows_sum(P[0]);
    const int j = j0 + cl;
    if (lane < 16 && j < n) {
      const double v = tot + a.c[p * n + j];
      rdv[j] = v;
      d2 += v * v;
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int i = lane + 64 * r;
    if (i < m) {
      const double v = ax[r] - a.b[p * m + i];
      rpv[i] = v;
      p2 += v * v;
    }
    if (i < k) {
      if (rzv) rzv[i] = gx[r] + s[i] - a.h[p * k + i];
      zs += z[i] * s[i];
    }
  }
  r3[0] = sqrt(ws64(d2));
  r3[1] = sqrt(ws64(p2));
  r3[2] = ws64(zs);
}

}  // namespace

// first step of the initial point: s = z = e (W = I at the setup), the
// right-hand side (-c, b, h, 0); every problem active, status maxit
__global__ __launch_bounds__(64) void socp_sqr_ipm_init_kernel(SqrIpmArgs a) {
  const int64_t p = blockIdx.x;
  const int lane = threadIdx.x, n = a.n, m = a.m, k = a.k;
  for (int i = lane; i < k; i += 64) {
    const double e = e_of(a.cones, i);
    a.s[p * k + i] = e;
    a.z[p * k + i] = e;
    a.dz[p * k + i] = a.h[p * k + i];
    a.ds[p * k + i] = 0.0;
  }
  for (int j = lane; j < n; j += 64) a.dx[p * n + j] = -a.c[p * n + j];
  for (int i = lane; i < m; i += 64) a.dy[p * m + i] = a.b[p * m + i];
  if (lane == 0) {
    a.active[p] = 1;
    a.status[p] = 1;  // maxit unless something else ends the solve
    a.iters[p] = 0;
  }
}

// the cone shift of the initial point (solver.jl:86-104): (x, y, iz) from the
// W = I solve; s = -iz (+ (1 + alpha_p) e), z = iz (+ (1 + alpha_d) e)
__global__ __launch_bounds__(64) void socp_sqr_ipm_shift_kernel(SqrIpmArgs a) {
  const int64_t p = blockIdx.x;
  const int lane = threadIdx.x, n = a.n, m = a.m, k = a.k;
  extern __shared__ double lds[];
  if (a.st_setup[p] != 0) {  // the W = I system is singular (the reference's `\` throws)
    if (lane == 0) {
      a.status[p] = a.st_setup[p];
      a.active[p] = 0;
      atomicSub(a.n_active, 1);  // the host stops launching once none is left
    }
    return;
  }
  double *iz = lds, *miz = lds + k;
  for (int i = lane; i < k; i += 64) {
    iz[i] = a.rz[p * k + i];
    miz[i] = -a.rz[p * k + i];
  }
  wsy();
  const double alphp = max_step_w(a.cones, miz, lane), alphd = max_step_w(a.cones, iz, lane);
  for (int i = lane; i < k; i += 64) {
    const double e = e_of(a.cones, i);
    a.s[p * k + i] = (fabs(alphp) < a.init_eps) ? -iz[i] : -iz[i] + (1.0 + alphp) * e;
    a.z[p * k + i] = (fabs(alphd) < a.init_eps) ? iz[i] : iz[i] + (1.0 + alphd) * e;
  }
  for (int j = lane; j < n; j += 64) a.x[p * n + j] = a.rx[p * n + j];
  for (int i = lane; i < m; i += 64) a.y[p * m + i] = a.ry[p * m + i];
}

// residuals, exit test and the affine right-hand side (solver.jl:106-125), after
// the setup launch: its status 4 is the scaling's DomainError (checked first,
// as compute_scaling runs first), 2 / 3 the factorisation's (after the exit test)
__global__ __launch_bounds__(64) void socp_sqr_ipm_resid_kernel(SqrIpmArgs a) {
  const int64_t p = blockIdx.x;
  if (!a.active[p]) return;
  const int lane = threadIdx.x, n = a.n, m = a.m, k = a.k;
  extern __shared__ double lds[];
  const int st = a.st_setup[p];
  if (st == SQR_DOMAIN) {
    if (lane == 0) {
      a.status[p] = SQR_DOMAIN;
      a.active[p] = 0;
      atomicSub(a.n_active, 1);  // the host stops launching once none is left
    }
    return;
  }
  double *lam = lds, *dsv = lds + k;
  const double* rec = a.rec + p * a.rec_stride;
  for (int i = lane; i < k; i += 64) lam[i] = rec[a.r_l + i];
  double r3[3];
  residuals_w(a, p, a.dx + p * n, a.dy + p * m, a.dz + p * k, r3, lane);
  vprod_w(a.cones, dsv, lam, lam, lane);
  if (lane == 0) {
    a.res[3 * p + 0] = r3[0];
    a.res[3 * p + 1] = r3[1];
    a.res[3 * p + 2] = r3[2];
  }
  if (r3[0] + r3[1] + r3[2] < a.tol) {
    if (lane == 0) {
      a.status[p] = 0;
      a.active[p] = 0;
      atomicSub(a.n_active, 1);  // the host stops launching once none is left
    }
    return;
  }
  if (st != 0) {  // cholesky! of H / S failed (PosDefException)
    if (lane == 0) {
      a.status[p] = st;
      a.active[p] = 0;
      atomicSub(a.n_active, 1);  // the host stops launching once none is left
    }
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup");  // this lane's own global writes above
  for (int j = lane; j < n; j += 64) a.dx[p * n + j] = -a.dx[p * n + j];
  for (int i = lane; i < m; i += 64) a.dy[p * m + i] = -a.dy[p * m + i];
  for (int i = lane; i < k; i += 64) {
    a.dz[p * k + i] = -a.dz[p * k + i];
    a.ds[p * k + i] = -dsv[i];
  }
}

// after the affine solve (solver.jl:128-140): kt3 = W rz, kt2 = W^-1 rs,
// t = compute_step, rho = 1 - t - t^2 (kt2'kt3) / (lam'lam), sigma =
// clamp(rho, 0, 1)^3, mu = lam'lam / deg; ds += sigma mu e - kt2 o kt3;
// dx, dy, dz *= 1 - sigma
__global__ __launch_bounds__(64) void socp_sqr_ipm_step1_kernel(SqrIpmArgs a) {
  const int64_t p = blockIdx.x;
  if (!a.active[p]) return;
  const int lane = threadIdx.x, n = a.n, m = a.m, k = a.k, nc = a.nc;
  extern __shared__ double lds[];
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
    return;
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
}

// after the combined solve (solver.jl:143-150): step = 0.99 compute_step, the update
__global__ __launch_bounds__(64) void socp_sqr_ipm_step2_kernel(SqrIpmArgs a, int it) {
  const int64_t p = blockIdx.x;
  if (!a.active[p]) return;
  const int lane = threadIdx.x, n = a.n, m = a.m, k = a.k, nc = a.nc;
  extern __shared__ double lds[];
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
    return;
  }
  const double stp = t * a.step;
  for (int j = lane; j < n; j += 64) a.x[p * n + j] += a.rx[p * n + j] * stp;
  for (int i = lane; i < m; i += 64) a.y[p * m + i] += a.ry[p * m + i] * stp;
  for (int i = lane; i < k; i += 64) {
    a.z[p * k + i] += rzv[i] * stp;
    a.s[p * k + i] += rsv[i] * stp;
  }
  if (lane == 0) a.iters[p] = it + 1;
}

// the exit quantities at the returned iterate (||rd||, ||rp||, z's) for every problem
__global__ __launch_bounds__(64) void socp_sqr_ipm_final_kernel(SqrIpmArgs a) {
  const int64_t p = blockIdx.x;
  const int lane = threadIdx.x;
  extern __shared__ double lds[];
  double r3[3];
  residuals_w(a, p, lds, lds + a.n, nullptr, r3, lane);
  if (lane == 0) {
    a.res[3 * p + 0] = r3[0];
    a.res[3 * p + 1] = r3[1];
    a.res[3 * p + 2] = r3[2];
  }
}

size_t sqr_ipm_lds_bytes(int n, int m, int k) {
  const int KP = (k + 1) / 2 * 2;
  size_t d = (size_t)7 * KP + MAXC;
  if ((size_t)(n + m) > d) d = (size_t)(n + m);
  return d * sizeof(double);
}

const void* sqr_ipm_kernel_ptr(int which) {
  switch (which) {
    case 0: return (const void*)socp_sqr_ipm_init_kernel;
    case 1: return (const void*)socp_sqr_ipm_shift_kernel;
    case 2: return (const void*)socp_sqr_ipm_resid_kernel;
    case 3: return (const void*)socp_sqr_ipm_step1_kernel;
    case 4: return (const void*)socp_sqr_ipm_step2_kernel;
    default: return (const void*)socp_sqr_ipm_final_kernel;
  }
}

}  // namespace socp
