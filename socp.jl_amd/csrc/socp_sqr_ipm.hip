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
#include "socp_sqr_step.hpp"

namespace socp {

namespace {

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
  extern __shared__ double lds[];
  ipm_step1_problem(a, p, lds, (int)threadIdx.x);
}

// after the combined solve (solver.jl:143-150): step = 0.99 compute_step, the update
__global__ __launch_bounds__(64) void socp_sqr_ipm_step2_kernel(SqrIpmArgs a, int it) {
  const int64_t p = blockIdx.x;
  if (!a.active[p]) return;
  extern __shared__ double lds[];
  ipm_step2_problem(a, p, it, lds, (int)threadIdx.x);
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
