// socp_sqr.hpp — launch interface of the rank-update KKT plugin (socp_sqr.hip):
// the reference's SqrScaling + SparseSolver (sqrscalings.jl, spsolver.jl).
#pragma once
#include <hip/hip_runtime.h>

#include "socp_small.hpp"  // ConeTable, MAXC, POC_K, SOC_K

namespace socp {

constexpr int SQR_NMAX = 64;   // n, m <= 64: one row per lane in the triangular solves (wavefront kernels)
constexpr int SQR_LMAX = 1024;  // n, m <= 1024: the workgroup kernels (factors packed in LDS, or in the
                                // record where they exceed it: SqrLayout::gfac)
constexpr int SQR_KMAX = 4096;  // k (and the vectors' LDS footprint <= 160 KiB)
constexpr int SQR_KC = 8;      // G rows per LDS chunk in the H product
constexpr int SQR_NW = 66;     // LDS row stride of a chunk (doubles; 16-byte aligned rows)
constexpr int SQR_RHS = 8;     // right-hand sides per forward sweep in L^-1 A'
constexpr int SQR_LT = 256;    // threads of a workgroup-kernel block (4 wavefronts)
constexpr int SQR_RC = 16;     // right-hand sides per chunk of C = L^-1 A' (workgroup kernels)
constexpr int SQR_CHOL_H = 2, SQR_CHOL_S = 3, SQR_DOMAIN = 4;  // include/socp.h status codes

struct SqrLayout {
  int large;     // 1: the workgroup kernels (n or m > SQR_NMAX)
  int gfac;      // 1 (large only): the packed factors and the C chunk in the record, not in LDS
  int ldl, ldm;  // LDS leading dimensions of C = L^-1 A' and L_S (odd: conflict-free row walks)
  // LDS offsets (doubles)
  int o_s, o_z, o_D, o_iW, o_u, o_v, o_l, o_wb, o_one, o_mu, o_rdgs, o_nv, o_mv, o_flag, o_X, o_S, total;
  // workgroup kernels: the two rank-1 chains' vectors, two more n-vectors, a
  // chunk of C, and the packed lower factor (L_H, then L_S, column-major)
  int o_w, o_wv, o_n0, o_n1, o_C, o_L;
  // per-problem factor record (doubles): L_H (n x n, column-major, zeros above
  // the diagonal), L_S (m x m), lambda, wb (k each), mu (nc), status; the
  // workgroup kernels add C = L^-1 A' (n x m, column-major) as scratch, and
  // with gfac the packed factors of H and S (r_P, r_PS) that LDS holds otherwise
  int64_t r_L, r_S, r_l, r_wb, r_mu, r_st, r_C, r_P, r_PS, rec;
};

// packed column-major lower triangle of an N x N matrix: element (i, j), i >= j
__host__ __device__ inline int sqr_pk(int i, int j, int N) { return j * (2 * N - j + 1) / 2 + (i - j); }

__host__ __device__ inline SqrLayout sqr_layout(int n, int m, int k, int nc) {
  SqrLayout L;
  L.large = (n > SQR_NMAX || m > SQR_NMAX) ? 1 : 0;
  L.ldl = n | 1;
  L.ldm = (m > 0 ? m : 1) | 1;
  const int KP = (k + 1) / 2 * 2;
  auto ev = [](int v) { return (v + 1) / 2 * 2; };
  const int NV = ev(n) > 64 ? ev(n) : 64, MV = ev(m) > 64 ? ev(m) : 64;
  int o = 0;
  L.o_s = o;    o += KP;
  L.o_z = o;    o += KP;
  L.o_D = o;    o += KP;
  L.o_iW = o;   o += KP;
  L.o_u = o;    o += KP;
  L.o_v = o;    o += KP;
  L.o_l = o;    o += KP;
  L.o_wb = o;   o += KP;
  L.o_one = o;  o += KP;
  L.o_mu = o;   o += MAXC;
  L.o_rdgs = o; o += MV;
  L.o_nv = o;   o += NV;
  L.o_mv = o;   o += MV;
  L.o_flag = o; o += 2;
  L.o_w = L.o_wv = L.o_n0 = L.o_n1 = L.o_C = L.o_L = 0;
  L.gfac = 0;
  if (!L.large) {
    L.o_X = o;
    int xs = 2 * SQR_KC * SQR_NW;          // Y row chunks (H product)
    if (xs < 64 * 17) xs = 64 * 17;        // the H tile transpose
    if (xs < m * L.ldl) xs = m * L.ldl;    // C = L^-1 A'
    o += ev(xs);
    L.o_S = o;    o += ev(m * L.ldm);
  } else {
    L.o_X = L.o_S = 0;
    L.o_w = o;  o += NV;
    L.o_wv = o; o += NV;
    L.o_n0 = o; o += NV;
    L.o_n1 = o; o += NV;
    const int th = n * (n + 1) / 2, ts = m * (m + 1) / 2;
    if ((int64_t)(o + ev(n * SQR_RC) + ev(th > ts ? th : ts)) * 8 <= 160 * 1024) {
      L.o_C = o;  o += ev(n * SQR_RC);
      L.o_L = o;  o += ev(th > ts ? th : ts);
    } else {
      L.gfac = 1;  // packed factors and the C chunk in the record (L1 / L2-cached)
    }
  }
  L.total = o;
  int64_t r = 0;
  L.r_L = r;  r += (int64_t)n * n;
  L.r_S = r;  r += (int64_t)m * m;
  L.r_l = r;  r += k;
  L.r_wb = r; r += k;
  L.r_mu = r; r += nc;
  L.r_st = r; r += 1;
  r = (r + 1) / 2 * 2;
  L.r_C = r;
  if (L.large) r += (int64_t)n * m;
  r = (r + 1) / 2 * 2;
  L.r_P = L.r_PS = r;
  if (L.gfac) {
    r += (int64_t)n * (n + 1) / 2;
    r = (r + 1) / 2 * 2;
    L.r_PS = r;
    r += (int64_t)m * (m + 1) / 2;
  }
  L.rec = (r + 1) / 2 * 2;
  return L;
}

struct SqrArgs {
  int64_t B;
  int n, m, k, nc;
  ConeTable cones;
  const double *A, *G;     // B x (m x n), B x (k x n), column-major per problem
  const uint8_t* sing;     // B (may be NULL)
  const double *s, *z;     // setup: B x k
  const double *dx, *dy, *dz, *ds;  // solve: right-hand sides
  double *cx, *cy, *cz, *cs;        // solve: solutions
  int32_t* status;         // B
  double* rec;             // B x rec
  unsigned long long* stamps;  // diagnostic build: per-phase cycle totals (setup kernel), else NULL
  const int32_t* active;   // B or NULL: problems with active[p] == 0 are skipped (the batched IPM's mask)
  int32_t init;            // solve: the initial-point system (solver.jl:68-84, an exact solve in the
                           // reference): m0 = -cy also when sing, as the dense kernel's MP_INIT
  // socp_sqr_solve_socp's iteration setup on the wavefront kernel (fuse_resid
  // != 0): the residuals (solver.jl:109-118) ride along the setup's pass over
  // G, and the resid kernel's exit test and affine right-hand side follow the
  // factorisation in the same launch (socp_sqr_ipm_resid_kernel's work)
  int32_t fuse_resid;
  const double *ix, *iy, *ic, *ib, *ih;  // the iterate's x, y and the data c, b, h
  double *odx, *ody, *odz, *ods, *ores;  // -rd, -rp, -rz, -lam o lam; ||rd||, ||rp||, z's
  int32_t *ostatus, *oactive, *n_active;
  double tol;
};

// the batched solve_socp on the rank-update plugin (socp_sqr_ipm.hip): the
// state, right-hand sides and KKT solutions of every problem, per-problem
// status / iteration count / activity, the setup launch's status
struct SqrIpmArgs {
  int64_t B;
  int n, m, k, nc, deg, sigma_exp;
  ConeTable cones;
  const double *A, *G, *c, *b, *h;
  const double* rec;  // the plugin's factor records: lambda, wb, mu at r_l, r_wb, r_mu
  int64_t rec_stride, r_l, r_wb, r_mu;
  double *x, *y, *z, *s, *dx, *dy, *dz, *ds, *rx, *ry, *rz, *rs, *res;
  int32_t *status, *iters, *active, *st_setup;
  int32_t* n_active;  // problems still iterating (decremented where active[p] is cleared)
  double tol, step, init_eps;
};
size_t sqr_ipm_lds_bytes(int n, int m, int k);
// The wavefront solve kernel reads no H-product chunk buffers: with
// SQR_SOLVE_TRIM its S block starts where they would (o_X), so its LDS is
// that much smaller (C2 shape: 19.9 -> 11.2 KB) and more waves fit a CU
#ifndef SQR_SOLVE_TRIM
#define SQR_SOLVE_TRIM 1
#endif
#ifndef SQR_SOLVE_WPE
#define SQR_SOLVE_WPE 3  // waves per SIMD the n = 64 solve kernel's registers allow (2: +7 % solve time)
#endif
__host__ __device__ inline SqrLayout sqr_solve_layout(int n, int m, int k, int nc) {
  SqrLayout L = sqr_layout(n, m, k, nc);
  if (SQR_SOLVE_TRIM && !L.large) {
    L.o_S = L.o_X;
    L.total = L.o_S + (m * L.ldm + 3) / 4 * 4;
  }
  return L;
}
// 0 init, 1 shift, 2 resid, 3 step1, 4 step2 (extra int argument: the iteration), 5 final
const void* sqr_ipm_kernel_ptr(int which);

// wavefront kernels for n, m <= SQR_NMAX (instantiation for n rounded up to
// 16), workgroup kernels (SQR_LT threads) above
const void* sqr_setup_kernel_ptr(int n, int m);
const void* sqr_solve_kernel_ptr(int n, int m);
// socp_sqr_solve_socp's two solves of an iteration with their step phases in
// one launch (wave shapes; nullptr for the workgroup shapes):
// kernel(SqrArgs solve, SqrIpmArgs ipm, int it)
const void* sqr_ipm_solves_kernel_ptr(int n, int m);
inline int sqr_block_threads(int n, int m) { return (n > SQR_NMAX || m > SQR_NMAX) ? SQR_LT : 64; }

}  // namespace socp
