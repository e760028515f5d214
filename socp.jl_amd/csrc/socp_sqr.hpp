// socp_sqr.hpp — launch interface of the rank-update KKT plugin (socp_sqr.hip):
// the reference's SqrScaling + SparseSolver (sqrscalings.jl, spsolver.jl).
#pragma once
#include <hip/hip_runtime.h>

#include "socp_small.hpp"  // ConeTable, MAXC, POC_K, SOC_K

namespace socp {

constexpr int SQR_NMAX = 64;   // n, m <= 64: one row per lane in the triangular solves
constexpr int SQR_KMAX = 256;  // k
constexpr int SQR_KC = 8;      // G rows per LDS chunk in the H product
constexpr int SQR_NW = 66;     // LDS row stride of a chunk (doubles; 16-byte aligned rows)
constexpr int SQR_RHS = 8;     // right-hand sides per forward sweep in L^-1 A'
constexpr int SQR_CHOL_H = 2, SQR_CHOL_S = 3, SQR_DOMAIN = 4;  // include/socp.h status codes

struct SqrLayout {
  int ldl, ldm;  // LDS leading dimensions of C = L^-1 A' and L_S (odd: conflict-free row walks)
  // LDS offsets (doubles)
  int o_s, o_z, o_D, o_iW, o_u, o_v, o_l, o_wb, o_one, o_mu, o_rdgs, o_nv, o_mv, o_flag, o_X, o_S, total;
  // per-problem factor record (doubles): L_H (n x n, column-major, zeros above
  // the diagonal), L_S (m x m), lambda, wb (k each), mu (nc), status
  int64_t r_L, r_S, r_l, r_wb, r_mu, r_st, rec;
};

__host__ __device__ inline SqrLayout sqr_layout(int n, int m, int k, int nc) {
  SqrLayout L;
  L.ldl = n | 1;
  L.ldm = (m > 0 ? m : 1) | 1;
  const int KP = (k + 1) / 2 * 2;
  auto ev = [](int v) { return (v + 1) / 2 * 2; };
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
  L.o_rdgs = o; o += 64;
  L.o_nv = o;   o += 64;
  L.o_mv = o;   o += 64;
  L.o_flag = o; o += 2;
  L.o_X = o;
  int xs = 2 * SQR_KC * SQR_NW;          // Y row chunks (H product)
  if (xs < 64 * 17) xs = 64 * 17;        // the H tile transpose
  if (xs < m * L.ldl) xs = m * L.ldl;    // C = L^-1 A'
  o += ev(xs);
  L.o_S = o;    o += ev(m * L.ldm);
  L.total = o;
  int64_t r = 0;
  L.r_L = r;  r += (int64_t)n * n;
  L.r_S = r;  r += (int64_t)m * m;
  L.r_l = r;  r += k;
  L.r_wb = r; r += k;
  L.r_mu = r; r += nc;
  L.r_st = r; r += 1;
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
};

const void* sqr_setup_kernel_ptr(int n);  // instantiation for n (rounded up to 16)
const void* sqr_solve_kernel_ptr(int n);

}  // namespace socp
