/*
 * socp_oracle.c — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference
 * dense SOCP path of BenChung/Socp.jl, used as the parity checker for the HIP
 * path and as the timed CPU baseline (`cpu_baseline.kind = "port"`).  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it;
 * the product (libsocp.so) never links or calls it.
 *
 * It follows the reference's op order, including the dense k x k product
 * iWiW = iW*iW' (scalings.jl:108), GWiWi = G'*iWiW and H = GWiWi*G
 * (densesolver.jl:42-43) and the explicit inverse Li = H^-1 through
 * potrs(I) (densesolver.jl:48).  LAPACK/BLAS calls are restated as the
 * reference-BLAS/LAPACK loop nests (dpotf2, dtrsm, dgemv); Julia runs
 * OpenBLAS or MKL there, so agreement is to rounding, not bitwise.
 *
 * The reference's DenseSolver does not run as written.  The
 * four minimal fixes applied here:
 *   densesolver.jl:48  `et`     -> ss.eyetgt (identity)
 *   densesolver.jl:49  `ss.ALi` -> ss.AtLi  (the field holding A*Li)
 *   densesolver.jl:50  `At`     -> pr.A'
 *   densesolver.jl:69,76 `ss.issng` -> the Problem's `sing` type parameter
 * Behaviour kept on purpose (bug-compatible):
 *   - the `sing` branch m0 = dy - cy (densesolver.jl:76-80) is reproduced as is;
 *   - the init shift applies (1+alpha)e even for alpha < 0 (solver.jl:91-101);
 *   - rho = 1 - t - t^2 (kt2.kt3)/(l.l) with the reference's minus sign (:132).
 * Failure semantics (the reference throws; we stop the problem and report):
 *   chol(H) fails -> status 2 (PosDefException, densesolver.jl:47)
 *   chol(S) fails -> status 3 (densesolver.jl:51)
 *   sqrt of a negative argument -> status 4 (Julia DomainError)
 *
 * Parity pinning: validated against every known-answer vector of
 * test/runtests.jl (see tests/golden/reference_kats.json and
 * tests/test_oracle.py).  The reference itself cannot run here (no Julia).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define EXPORT __attribute__((visibility("default")))

enum { POC = 0, SOC = 1 };

typedef struct {
  int ncones;
  const int32_t* kind;
  const int32_t* offs;
  const int32_t* dim;
} cones_t;

/* Julia semantics: sqrt(x<0) throws DomainError; min/max propagate NaN. */
static inline double jsqrt(double x, int* dom) {
  if (x < 0.0) *dom = 1;
  return sqrt(x);
}
static inline double jmin(double a, double b) {
  if (isnan(a) || isnan(b)) return NAN;
  return a < b ? a : b;
}
static inline double jmax(double a, double b) {
  if (isnan(a) || isnan(b)) return NAN;
  return a > b ? a : b;
}

/* ---------------- vectors.jl ---------------- */

/* make_e! (vectors.jl:7-24) */
static void make_e(const cones_t* C, double* r) {
  for (int c = 0; c < C->ncones; ++c) {
    int o = C->offs[c], d = C->dim[c];
    if (C->kind[c] == POC) {
      for (int i = 0; i < d; ++i) r[o + i] = 1.0;
    } else {
      r[o] = 1.0;
      for (int i = 1; i < d; ++i) r[o + i] = 0.0;
    }
  }
}

/* vprod! (vectors.jl:58-81): Jordan product t = u o v */
static void vprod(const cones_t* C, double* t, const double* u, const double* v) {
  for (int c = 0; c < C->ncones; ++c) {
    int o = C->offs[c], d = C->dim[c];
    if (C->kind[c] == POC) {
      for (int i = 0; i < d; ++i) t[o + i] = u[o + i] * v[o + i];
    } else {
      double t0 = 0.0;
      for (int i = 0; i < d; ++i) t0 += u[o + i] * v[o + i];
      double iu = u[o], iv = v[o];
      t[o] = t0;
      for (int i = 1; i < d; ++i) t[o + i] = iu * v[o + i] + iv * u[o + i];
    }
  }
}

/* iprod! (vectors.jl:99-125): t = lam^-1 o v, SOC via the O(d^2) loop */
static void iprod(const cones_t* C, double* t, const double* lam, const double* v) {
  for (int c = 0; c < C->ncones; ++c) {
    int o = C->offs[c], d = C->dim[c];
    if (C->kind[c] == POC) {
      for (int i = 0; i < d; ++i) t[o + i] = v[o + i] / lam[o + i];
    } else {
      double l1 = lam[o];
      double a = l1 * l1;
      for (int i = 1; i < d; ++i) a -= lam[o + i] * lam[o + i];
      for (int i = 0; i < d; ++i) t[o + i] = 0.0;
      t[o] += v[o] * l1 / a;
      for (int j = 1; j < d; ++j) t[o] -= v[o + j] * lam[o + j] / a;
      for (int i = 1; i < d; ++i) {
        t[o + i] -= v[o] * lam[o + i] / a;
        for (int j = 1; j < d; ++j)
          t[o + i] += v[o + j] * ((i == j ? a : 0.0) + lam[o + i] * lam[o + j]) / (l1 * a);
      }
    }
  }
}

/* cgt (vectors.jl:136-161) */
static int cgt(const cones_t* C, const double* x, const double* dx) {
  for (int c = 0; c < C->ncones; ++c) {
    int o = C->offs[c], d = C->dim[c];
    if (C->kind[c] == POC) {
      for (int i = 0; i < d; ++i)
        if (x[o + i] + dx[o + i] < 0) return 0;
    } else {
      double tot = 0.0;
      for (int i = 1; i < d; ++i) {
        double val = x[o + i] + dx[o + i];
        tot += val * val;
      }
      if (!(sqrt(tot) <= x[o] + dx[o])) return 0;
    }
  }
  return 1;
}

/* deg (vectors.jl:165-179) */
static int deg(const cones_t* C) {
  int dg = 0;
  for (int c = 0; c < C->ncones; ++c) dg += (C->kind[c] == POC) ? C->dim[c] : 1;
  return dg;
}

/* ---------------- mats.jl ---------------- */

/* max_step (mats.jl:1-28) */
static double max_step(const cones_t* C, const double* x) {
  double maxim = -INFINITY;
  for (int c = 0; c < C->ncones; ++c) {
    int o = C->offs[c], d = C->dim[c];
    double val;
    if (C->kind[c] == POC) {
      double minim = INFINITY;
      for (int i = 0; i < d; ++i)
        if (x[o + i] < minim) minim = x[o + i];
      val = -minim;
    } else {
      double sq = 0.0;
      for (int i = 1; i < d; ++i) sq += x[o + i] * x[o + i];
      val = sqrt(sq) - x[o];
    }
    if (val > maxim) maxim = val;
  }
  return maxim;
}

/* scmax (mats.jl:42-86) */
static double scmax(const cones_t* C, const double* li, const double* xi, int* dom) {
  double mxv = -INFINITY;
  for (int c = 0; c < C->ncones; ++c) {
    int o = C->offs[c], d = C->dim[c];
    double val;
    if (C->kind[c] == POC) {
      val = -INFINITY;
      for (int i = 0; i < d; ++i) {
        double v = -xi[o + i] / li[o + i];
        if (v > val) val = v;
      }
    } else {
      double ai = li[o] * li[o];
      for (int i = 1; i < d; ++i) ai -= li[o + i] * li[o + i];
      double a = 1.0 / jsqrt(ai, dom);
      double r1 = a * li[o] * xi[o];
      for (int i = 1; i < d; ++i) r1 -= a * li[o + i] * xi[o + i];
      double cst = (r1 + xi[o]) / (a * li[o] + 1.0);
      double r2s = 0.0;
      for (int i = 1; i < d; ++i) {
        double q = a * (xi[o + i] - cst * a * li[o + i]);
        r2s += q * q;
      }
      val = sqrt(r2s) - a * r1;
    }
    if (val > mxv) mxv = val;
  }
  return mxv;
}

/* compute_step (mats.jl:30-40) */
static double compute_step(const cones_t* C, const double* l, const double* ds, const double* dz,
                           int* dom) {
  double mxs = scmax(C, l, ds, dom);
  double mxz = scmax(C, l, dz, dom);
  double t = jmax(jmax(mxs, mxz), 0.0);
  if (t == 0.0) return 1.0;
  return jmin(1.0, 1.0 / t);
}

/* ---------------- scalings.jl ---------------- */

typedef struct {
  int k;
  double *W, *iW, *iWiW; /* k x k column-major, zero outside the cone blocks */
  double* l;             /* lambda */
  double* mu;            /* per cone */
  double* wbs;           /* sqrt(s/z) for POC, wbar for SOC */
  double *sik, *zik;
} scaling_t;

#define M(A, ld, i, j) (A)[(size_t)(j) * (ld) + (i)]

/* compute_scaling (scalings.jl:22-110) */
static void compute_scaling_x(const cones_t* C, scaling_t* S, const double* s, const double* z,
                              int* dom, int structured);
static void compute_scaling(const cones_t* C, scaling_t* S, const double* s, const double* z,
                            int* dom) {
  compute_scaling_x(C, S, s, z, dom, 0);
}
static void compute_scaling_x(const cones_t* C, scaling_t* S, const double* s, const double* z,
                              int* dom, int structured) {
  int k = S->k;
  for (int c = 0; c < C->ncones; ++c) {
    int o = C->offs[c], dim = C->dim[c];
    if (C->kind[c] == POC) {
      for (int i = 0; i < dim; ++i) {
        int ii = o + i;
        M(S->W, k, ii, ii) = jsqrt(s[ii] / z[ii], dom);
        M(S->iW, k, ii, ii) = jsqrt(z[ii] / s[ii], dom);
        S->l[ii] = jsqrt(s[ii] * z[ii], dom);
        S->wbs[ii] = jsqrt(s[ii] / z[ii], dom);
      }
      continue;
    }
    double *sik = S->sik, *zik = S->zik;
    for (int i = 0; i < dim; ++i) {
      sik[i] = s[o + i];
      zik[i] = z[o + i];
    }
    double onrmz = zik[0] * zik[0];
    double onrms = sik[0] * sik[0];
    for (int i = 1; i < dim; ++i) {
      onrmz -= zik[i] * zik[i];
      onrms -= sik[i] * sik[i];
    }
    double nrmz = jsqrt(onrmz, dom);
    double nrms = jsqrt(onrms, dom);
    double fz = 1.0 / nrmz, fs = 1.0 / nrms;
    for (int i = 0; i < dim; ++i) zik[i] *= fz;
    for (int i = 0; i < dim; ++i) sik[i] *= fs;
    double nsum = 0.0;
    for (int i = 0; i < dim; ++i) nsum += zik[i] * sik[i];
    double gamma = jsqrt((1.0 + nsum) / 2.0, dom);
    double* wb = S->wbs + o;
    wb[0] = sik[0] + zik[0];
    for (int i = 1; i < dim; ++i) wb[i] = sik[i] - zik[i];
    double fg = 1.0 / (2.0 * gamma);
    for (int i = 0; i < dim; ++i) wb[i] *= fg;
    int bl = dim - 1;
    double denom = wb[0] + 1.0;
    double mu = jsqrt(nrms / nrmz, dom);
    S->mu[c] = mu;
    if (!structured)
    for (int j = 1; j <= bl; ++j)
      for (int i = 1; i <= bl; ++i) {
        double cellv = ((i == j) ? 1.0 : 0.0) + wb[i] * wb[j] / denom;
        M(S->W, k, o + i, o + j) = cellv * mu;
        M(S->iW, k, o + i, o + j) = cellv / mu;
      }
    if (!structured) {
      for (int i = 0; i < dim; ++i) M(S->W, k, o, o + i) = wb[i] * mu;
      M(S->iW, k, o, o) = wb[0] / mu;
      for (int i = 1; i < dim; ++i) {
        M(S->W, k, o + i, o) = wb[i] * mu;
        M(S->iW, k, o, o + i) = -wb[i] / mu;
        M(S->iW, k, o + i, o) = -wb[i] / mu;
      }
    }
    double ziv = zik[0], siv = sik[0];
    double tmv1 = jsqrt(nrms * nrmz, dom);
    double mult = tmv1 / (ziv + siv + 2.0 * gamma);
    double gs = gamma + ziv, gz = gamma + siv;
    for (int i = 0; i < dim; ++i) sik[i] *= gs;
    for (int i = 0; i < dim; ++i) zik[i] *= gz;
    for (int i = 1; i < dim; ++i) S->l[o + i] = (sik[i] + zik[i]) * mult;
    S->l[o] = gamma * tmv1;
  }
  /* iWiW = iW * iW' (scalings.jl:108): dense k^3 GEMM as the reference does
     (the structured mode applies W^-1 per cone instead and never forms it) */
  if (structured) return;
  for (int j = 0; j < k; ++j)
    for (int i = 0; i < k; ++i) {
      double acc = 0.0;
      for (int q = 0; q < k; ++q) acc += M(S->iW, k, i, q) * M(S->iW, k, j, q);
      M(S->iWiW, k, i, j) = acc;
    }
}

/* scale! = W*x, iscale! = W^-1*x (scalings.jl:112-173) */
static void scale_w(const cones_t* C, const scaling_t* S, const double* x, double* op) {
  const double* wb = S->wbs;
  for (int c = 0; c < C->ncones; ++c) {
    int o = C->offs[c], d = C->dim[c];
    if (C->kind[c] == POC) {
      for (int i = o; i < o + d; ++i) op[i] = wb[i] * x[i];
    } else {
      double mu = S->mu[c], del = 0.0;
      for (int i = o + 1; i < o + d; ++i) del += wb[i] * x[i];
      double cst = (x[o] + del / (1.0 + wb[o]));
      op[o] = mu * (wb[o] * x[o] + del);
      for (int i = o + 1; i < o + d; ++i) op[i] = mu * (x[i] + cst * wb[i]);
    }
  }
}
static void iscale_w(const cones_t* C, const scaling_t* S, const double* x, double* op) {
  const double* wb = S->wbs;
  for (int c = 0; c < C->ncones; ++c) {
    int o = C->offs[c], d = C->dim[c];
    if (C->kind[c] == POC) {
      for (int i = o; i < o + d; ++i) op[i] = 1.0 / wb[i] * x[i];
    } else {
      double mu = S->mu[c], del = 0.0;
      for (int i = o + 1; i < o + d; ++i) del += wb[i] * x[i];
      double cst = (-x[o] + del / (1.0 + wb[o]));
      op[o] = 1.0 / mu * (wb[o] * x[o] - del);
      for (int i = o + 1; i < o + d; ++i) op[i] = 1.0 / mu * (x[i] + cst * wb[i]);
    }
  }
}

/* ---------------- LAPACK restatements ---------------- */

/* dpotf2('U'): A = U'U in the upper triangle; returns 0 or j+1 on failure. */
static int potrf_u(double* A, int n) {
  for (int j = 0; j < n; ++j) {
    double dot = 0.0;
    for (int q = 0; q < j; ++q) dot += M(A, n, q, j) * M(A, n, q, j);
    double ajj = M(A, n, j, j) - dot;
    if (ajj <= 0.0 || isnan(ajj)) {
      M(A, n, j, j) = ajj;
      return j + 1;
    }
    ajj = sqrt(ajj);
    M(A, n, j, j) = ajj;
    double r = 1.0 / ajj;
    for (int jj = j + 1; jj < n; ++jj) {
      double t = 0.0;
      for (int q = 0; q < j; ++q) t += M(A, n, q, j) * M(A, n, q, jj);
      M(A, n, j, jj) = (M(A, n, j, jj) - t) * r;
    }
  }
  return 0;
}

/* dpotrs('U') for one column: solve U'U x = b in place (dtrsm 'L','U','T' then 'L','U','N'). */
static void potrs_u(const double* U, int n, double* b) {
  for (int i = 0; i < n; ++i) {
    double t = b[i];
    for (int q = 0; q < i; ++q) t -= M(U, n, q, i) * b[q];
    b[i] = t / M(U, n, i, i);
  }
  for (int q = n - 1; q >= 0; --q) {
    if (b[q] != 0.0) {
      b[q] /= M(U, n, q, q);
      for (int i = 0; i < q; ++i) b[i] -= b[q] * M(U, n, i, q);
    }
  }
}

/* ---------------- densesolver.jl ---------------- */

typedef struct {
  int n, m, k, sing;
  int structured;        /* OR_F_STRUCTURED: the build's algorithm, not the reference op order */
  int cholsolve;         /* OR_F_CHOLSOLVE (with structured): no explicit Li -- Z = U^-T A' kept in
                            ALi (as Z', m x n), S = Z'Z, Li v by the two triangular solves of potrs
                            (the register kernel's order for m <= 16) */
  int inv_yty;           /* OR_F_INV_YTY (with structured, without cholsolve): Li = Y'Y with
                            Y = U^-T = L^-1 formed by forward substitution against I (potri's
                            order, the kernels' explicit inverse) instead of potrs(I) */
  const cones_t* C;
  const double *A, *G; /* column-major m x n, k x n */
  double *AA, *GWiWi, *H, *Li, *ALi, *S, *Y;
  double *k0, *k1, *k2, *m0, *n0, *n1;
} dense_t;

/* setup_iter(::DenseSolver) (densesolver.jl:41-52, with the fixes); returns 0/2/3 */
static void iscale_w(const cones_t* C, const scaling_t* S, const double* x, double* op);
static int setup_iter(dense_t* D, const scaling_t* S) {
  int n = D->n, m = D->m, k = D->k;
  if (D->structured) {
    /* X = W^-1 G column by column (iscale!, O(k) per column), H = X'X (one
       triangle, mirrored): the reference's iWiW GEMM, G'*iWiW and *G done
       structurally -- the algorithm the MI355X kernels run.  X is kept in the
       GWiWi buffer (k x n, column-major). */
    double* X = D->GWiWi;
    for (int a = 0; a < n; ++a) iscale_w(D->C, S, D->G + (size_t)a * k, X + (size_t)a * k);
    for (int b = 0; b < n; ++b)
      for (int a = 0; a <= b; ++a) {
        double acc = 0.0;
        for (int i = 0; i < k; ++i) acc += X[(size_t)a * k + i] * X[(size_t)b * k + i];
        M(D->H, n, a, b) = acc;
        M(D->H, n, b, a) = acc;
      }
  } else {
  for (int j = 0; j < k; ++j)
    for (int a = 0; a < n; ++a) {
      double acc = 0.0;
      for (int i = 0; i < k; ++i) acc += M(D->G, k, i, a) * M(S->iWiW, k, i, j);
      M(D->GWiWi, n, a, j) = acc;
    }
  for (int b = 0; b < n; ++b)
    for (int a = 0; a < n; ++a) {
      double acc = 0.0;
      for (int i = 0; i < k; ++i) acc += M(D->GWiWi, n, a, i) * M(D->G, k, i, b);
      M(D->H, n, a, b) = acc;
    }
  }
  if (D->sing)
    for (size_t q = 0; q < (size_t)n * n; ++q) D->H[q] += D->AA[q];
  if (potrf_u(D->H, n)) return 2;
  if (D->cholsolve) {
    /* H = U'U: Z = U^-T A' column by column (Z' in ALi), S = Z'Z */
    for (int r = 0; r < m; ++r) {
      double* zr = D->n1; /* scratch */
      for (int a = 0; a < n; ++a) {
        double t = M(D->A, m, r, a);
        for (int q = 0; q < a; ++q) t -= M(D->H, n, q, a) * zr[q];
        zr[a] = t / M(D->H, n, a, a);
      }
      for (int a = 0; a < n; ++a) M(D->ALi, m, r, a) = zr[a];
    }
    for (int q = 0; q < m; ++q)
      for (int r = 0; r < m; ++r) {
        double acc = 0.0;
        for (int a = 0; a < n; ++a) acc += M(D->ALi, m, r, a) * M(D->ALi, m, q, a);
        M(D->S, m, r, q) = acc;
      }
    if (potrf_u(D->S, m)) return 3;
    return 0;
  }
  if (D->inv_yty) {
    /* Y = U^-T = L^-1 (lower), column j by forward substitution U'y = e_j */
    double* Y = D->Y;
    for (int j = 0; j < n; ++j) {
      double* y = Y + (size_t)j * n;
      for (int i = 0; i < n; ++i) {
        double t = (i == j) ? 1.0 : 0.0;
        for (int q = j; q < i; ++q) t -= M(D->H, n, q, i) * y[q];
        y[i] = (i < j) ? 0.0 : t / M(D->H, n, i, i);
      }
    }
    /* Li = Y'Y: Li[a][b] = sum_{q >= max(a, b)} Y[q][a] Y[q][b] */
    for (int b = 0; b < n; ++b)
      for (int a = 0; a < n; ++a) {
        double acc = 0.0;
        for (int q = (a > b ? a : b); q < n; ++q) acc += Y[(size_t)a * n + q] * Y[(size_t)b * n + q];
        M(D->Li, n, a, b) = acc;
      }
  } else
  /* Li = H^-1 via ldiv!(Li, fact, I) */
  for (int j = 0; j < n; ++j) {
    double* col = D->Li + (size_t)j * n;
    for (int i = 0; i < n; ++i) col[i] = (i == j) ? 1.0 : 0.0;
    potrs_u(D->H, n, col);
  }
  for (int b = 0; b < n; ++b)
    for (int r = 0; r < m; ++r) {
      double acc = 0.0;
      for (int a = 0; a < n; ++a) acc += M(D->A, m, r, a) * M(D->Li, n, a, b);
      M(D->ALi, m, r, b) = acc;
    }
  for (int q = 0; q < m; ++q)
    for (int r = 0; r < m; ++r) {
      double acc = 0.0;
      for (int a = 0; a < n; ++a) acc += M(D->ALi, m, r, a) * M(D->A, m, q, a);
      M(D->S, m, r, q) = acc;
    }
  if (potrf_u(D->S, m)) return 3;
  return 0;
}

/* solve_kkt(::DenseSolver) (densesolver.jl:54-90); `init` selects the exact
 * elimination (m0 = -cy) used for the W = I initial-point system. */
static void solve_kkt(dense_t* D, const cones_t* C, const scaling_t* S, const double* dx,
                      const double* dy, const double* dz, const double* ds, double* cx, double* cy,
                      double* cz, double* cs) {
  int n = D->n, m = D->m, k = D->k;
  iprod(C, D->k0, S->l, ds);
  scale_w(C, S, D->k0, D->k1);
  for (int i = 0; i < k; ++i) D->k2[i] = dz[i] - D->k1[i];
  if (D->structured) {
    /* G'W^-1W^-1 k2 = X'(W^-1 k2) */
    iscale_w(C, S, D->k2, cz);
    for (int a = 0; a < n; ++a) {
      double acc = 0.0;
      for (int i = 0; i < k; ++i) acc += D->GWiWi[(size_t)a * k + i] * cz[i];
      D->n0[a] = acc;
    }
  } else
  for (int a = 0; a < n; ++a) {
    double acc = 0.0;
    for (int i = 0; i < k; ++i) acc += M(D->GWiWi, n, a, i) * D->k2[i];
    D->n0[a] = acc;
  }
  for (int a = 0; a < n; ++a) D->n0[a] += dx[a];
  if (D->sing)
    for (int a = 0; a < n; ++a) {
      double acc = 0.0;
      for (int r = 0; r < m; ++r) acc += M(D->A, m, r, a) * dy[r];
      D->n0[a] += acc;
    }
  if (D->cholsolve) /* t = U^-T n0 (the first half of potrs); A Li n0 = Z't */
    for (int i = 0; i < n; ++i) {
      double t = D->n0[i];
      for (int q = 0; q < i; ++q) t -= M(D->H, n, q, i) * D->n0[q];
      D->n0[i] = t / M(D->H, n, i, i);
    }
  for (int r = 0; r < m; ++r) {
    double acc = 0.0;
    for (int a = 0; a < n; ++a) acc += M(D->ALi, m, r, a) * D->n0[a];
    D->m0[r] = acc;
  }
  for (int r = 0; r < m; ++r) D->m0[r] -= dy[r];
  for (int r = 0; r < m; ++r) cy[r] = D->m0[r];
  potrs_u(D->S, m, cy);
  if (D->sing)
    for (int r = 0; r < m; ++r) D->m0[r] = dy[r] - cy[r];
  else
    for (int r = 0; r < m; ++r) D->m0[r] = -cy[r];
  if (D->cholsolve) {
    /* cx = U^-1 (t + Z m0) (the second half of potrs) */
    for (int a = 0; a < n; ++a) {
      double acc = 0.0;
      for (int r = 0; r < m; ++r) acc += M(D->ALi, m, r, a) * D->m0[r];
      cx[a] = D->n0[a] + acc;
    }
    for (int q = n - 1; q >= 0; --q) {
      double t = cx[q];
      for (int i = q + 1; i < n; ++i) t -= M(D->H, n, q, i) * cx[i];
      cx[q] = t / M(D->H, n, q, q);
    }
  } else {
  for (int a = 0; a < n; ++a) {
    double acc = 0.0;
    for (int r = 0; r < m; ++r) acc += M(D->A, m, r, a) * D->m0[r];
    D->n1[a] = acc;
  }
  for (int a = 0; a < n; ++a) D->n0[a] += D->n1[a];
  for (int a = 0; a < n; ++a) {
    double acc = 0.0;
    for (int b = 0; b < n; ++b) acc += M(D->Li, n, a, b) * D->n0[b];
    cx[a] = acc;
  }
  }
  for (int i = 0; i < k; ++i) {
    double acc = 0.0;
    for (int a = 0; a < n; ++a) acc += M(D->G, k, i, a) * cx[a];
    D->k1[i] = acc;
  }
  for (int i = 0; i < k; ++i) D->k1[i] -= D->k2[i];
  if (D->structured) {
    /* iWiW k1 = W^-1 (W^-1 k1); cs (written last) is the scratch */
    iscale_w(C, S, D->k1, cs);
    iscale_w(C, S, cs, cz);
  } else
  for (int i = 0; i < k; ++i) {
    double acc = 0.0;
    for (int q = 0; q < k; ++q) acc += M(S->iWiW, k, i, q) * D->k1[q];
    cz[i] = acc;
  }
  scale_w(C, S, cz, D->k1);
  for (int i = 0; i < k; ++i) D->k0[i] -= D->k1[i];
  scale_w(C, S, D->k0, cs);
}

/* ---------------- sqrscalings.jl + spsolver.jl (the rank-update path) ----------------
 *
 * SqrScaling (sqrscalings.jl:8-139): W^-2 = D + u u' - v v' per SOC cone, D
 * diagonal.  SparseSolver (spsolver.jl:60-130): H = G'DG (+A'A if sing) is
 * factored, then one rank-1 update with G'u and one downdate with G'v per SOC
 * cone (modify_factors!, sqrscalings.jl:160-194), S = (L^-1 A')'(L^-1 A') is
 * factored, and solve_kkt applies H^-1 and S^-1 by triangular solves.
 *
 * The reference runs this through CHOLMOD (SuiteSparse, the Julia stdlib's
 * SuiteSparse.CHOLMOD: a fill-reducing permutation P, supernodal LDL'/LL',
 * lowrankupdowndate! = the Davis-Hager rank-1 modification).  CHOLMOD is not
 * part of /root/reference; restated here as the textbook algorithms on the
 * dense lower factor, without the permutation: the factor of P H P' and H
 * give the same solves to rounding.  A rank-1 update computes, column by
 * column, r = sqrt(L_jj^2 + sig w_j^2), c = r / L_jj, s = w_j / L_jj,
 * L_ij = (L_ij + sig s w_i) / c, w_i = c w_i - s L_ij (i > j); a downdate with
 * r^2 <= 0 is a loss of positive definiteness -> status 2, as cholesky! of H.
 * Pinned by runtests.jl:50-93 (the factor after modify_factors! inverts to the
 * dense H^-1) and :95-128 (the KKT golden, produced on this path). */

typedef struct {
  double *D, *iWd, *u, *v; /* k each: diag of iWiW and iW; u, v of every SOC cone (disjoint supports) */
} sqr_t;

/* compute_scaling(::SqrScaling) (sqrscalings.jl:50-58 POC, :66-139 SOC), op order kept */
static void sqr_compute_scaling(const cones_t* C, scaling_t* S, sqr_t* Q, const double* s,
                                const double* z, int* dom) {
  for (int c = 0; c < C->ncones; ++c) {
    int o = C->offs[c], dim = C->dim[c];
    if (C->kind[c] == POC) {
      for (int ii = o; ii < o + dim; ++ii) {
        Q->D[ii] = z[ii] / s[ii];
        Q->iWd[ii] = jsqrt(z[ii] / s[ii], dom);
        S->l[ii] = jsqrt(s[ii] * z[ii], dom);
        S->wbs[ii] = jsqrt(s[ii] / z[ii], dom);
        Q->u[ii] = 0.0;
        Q->v[ii] = 0.0;
      }
      continue;
    }
    double *sbk = S->sik, *zbk = S->zik;
    for (int i = 0; i < dim; ++i) {
      sbk[i] = s[o + i];
      zbk[i] = z[o + i];
    }
    double sprod = sbk[0] * sbk[0], zprod = zbk[0] * zbk[0];
    for (int i = 1; i < dim; ++i) sprod -= sbk[i] * sbk[i];
    for (int i = 1; i < dim; ++i) zprod -= zbk[i] * zbk[i];
    double fs = 1.0 / jsqrt(sprod, dom), fz = 1.0 / jsqrt(zprod, dom);
    for (int i = 0; i < dim; ++i) sbk[i] *= fs;
    for (int i = 0; i < dim; ++i) zbk[i] *= fz;
    double nsum = 0.0;
    for (int i = 0; i < dim; ++i) nsum += zbk[i] * sbk[i];
    double gamma = jsqrt((1.0 + nsum) / 2.0, dom);
    double* wb = S->wbs + o;
    wb[0] = (sbk[0] + zbk[0]) / (2.0 * gamma);
    for (int i = 1; i < dim; ++i) wb[i] = (sbk[i] - zbk[i]) / (2.0 * gamma);
    S->mu[c] = jsqrt(jsqrt(sprod / zprod, dom), dom);
    double inusq = 1.0 / jsqrt(sprod / zprod, dom);
    double inu = 1.0 / jsqrt(jsqrt(sprod / zprod, dom), dom);
    double wb0 = wb[0], wb1sq = 0.0;
    for (int i = 1; i < dim; ++i) wb1sq += wb[i] * wb[i];
    double cv = -(1.0 + wb0 + wb1sq / (1.0 + wb0));
    double d = 1.0 + 2.0 / (1.0 + wb0) + wb1sq / ((1.0 + wb0) * (1.0 + wb0));
    double a = (wb0 * wb0 + wb1sq - cv * cv * wb1sq / (1.0 + d * wb1sq)) / 2.0;
    double u0 = jsqrt(wb0 * wb0 + wb1sq - a, dom);
    double u1 = cv / u0;
    double v1 = jsqrt(cv * cv / (u0 * u0) - d, dom);
    Q->D[o] = a * inusq;
    Q->iWd[o] = sqrt(fabs(a * inusq));
    for (int i = 1; i < dim; ++i) {
      Q->D[o + i] = inusq;
      Q->iWd[o + i] = jsqrt(inusq, dom);
    }
    Q->u[o] = inu * u0;
    Q->v[o] = 0.0;
    for (int i = 1; i < dim; ++i) {
      double wbv = inu * wb[i];
      Q->u[o + i] = u1 * wbv;
      Q->v[o + i] = v1 * wbv;
    }
    double ziv = zbk[0], siv = sbk[0];
    double tmv1 = jsqrt(jsqrt(sprod, dom) * jsqrt(zprod, dom), dom);
    double mult = tmv1 / (ziv + siv + 2.0 * gamma);
    for (int i = 1; i < dim; ++i) S->l[o + i] = (sbk[i] * (gamma + ziv) + zbk[i] * (gamma + siv)) * mult;
    S->l[o] = gamma * tmv1;
  }
}

/* dense lower Cholesky (column by column, left-looking); 0 or j+1 at a failed pivot */
static int potrf_l(double* L, int n) {
  for (int j = 0; j < n; ++j) {
    double ajj = M(L, n, j, j);
    for (int q = 0; q < j; ++q) ajj -= M(L, n, j, q) * M(L, n, j, q);
    if (ajj <= 0.0 || isnan(ajj)) return j + 1;
    ajj = sqrt(ajj);
    M(L, n, j, j) = ajj;
    for (int i = j + 1; i < n; ++i) {
      double t = M(L, n, i, j);
      for (int q = 0; q < j; ++q) t -= M(L, n, i, q) * M(L, n, j, q);
      M(L, n, i, j) = t / ajj;
    }
    for (int i = 0; i < j; ++i) M(L, n, i, j) = 0.0;
  }
  return 0;
}

/* L L' +/- w w' (sig = +1 update, -1 downdate); w is overwritten; 0 or j+1 */
static int chol_rank1(double* L, int n, double* w, double sig) {
  for (int j = 0; j < n; ++j) {
    double ljj = M(L, n, j, j), wj = w[j];
    double r2 = ljj * ljj + sig * wj * wj;
    if (r2 <= 0.0 || isnan(r2)) return j + 1;
    double r = sqrt(r2);
    double c = r / ljj, s = wj / ljj;
    M(L, n, j, j) = r;
    for (int i = j + 1; i < n; ++i) {
      double lij = (M(L, n, i, j) + sig * s * w[i]) / c;
      M(L, n, i, j) = lij;
      w[i] = c * w[i] - s * lij;
    }
  }
  return 0;
}

/* L y = b, then L' x = y, in place */
static void chol_solve_l(const double* L, int n, double* b) {
  for (int j = 0; j < n; ++j) {
    b[j] /= M(L, n, j, j);
    for (int i = j + 1; i < n; ++i) b[i] -= M(L, n, i, j) * b[j];
  }
  for (int j = n - 1; j >= 0; --j) {
    double t = b[j];
    for (int i = j + 1; i < n; ++i) t -= M(L, n, i, j) * b[i];
    b[j] = t / M(L, n, j, j);
  }
}

/* setup_iter(::SparseSolver) (spsolver.jl:60-84).  L_H in D->H, L_S in D->S,
 * C = L^-1 A' (n x m) in D->ALi.  Returns 0 / 2 (chol of H or a downdate) / 3. */
static int sqr_setup_iter(dense_t* D, const cones_t* C, const sqr_t* Q) {
  int n = D->n, m = D->m, k = D->k;
  double* L = D->H;
  for (int b = 0; b < n; ++b)
    for (int a = 0; a < n; ++a) {
      double acc = 0.0;
      if (!D->sing) /* GiW = iW G' -> factor of (iW G)'(iW G) (:62-64) */
        for (int i = 0; i < k; ++i) acc += (Q->iWd[i] * M(D->G, k, i, a)) * (Q->iWd[i] * M(D->G, k, i, b));
      else /* Gint = iWiW G; i1 = G' Gint + AA (:67-71) */
        for (int i = 0; i < k; ++i) acc += M(D->G, k, i, a) * (Q->D[i] * M(D->G, k, i, b));
      M(L, n, a, b) = acc + (D->sing ? M(D->AA, n, a, b) : 0.0);
    }
  if (potrf_l(L, n)) return 2;
  /* modify_factors! (sqrscalings.jl:160-194): per SOC cone, +G'u then -G'v */
  double* w = D->n1;
  for (int c = 0; c < C->ncones; ++c) {
    if (C->kind[c] != SOC) continue;
    int o = C->offs[c], d = C->dim[c];
    for (int pass = 0; pass < 2; ++pass) {
      const double* uv = pass ? Q->v : Q->u;
      for (int a = 0; a < n; ++a) {
        double acc = 0.0;
        for (int i = o; i < o + d; ++i) acc += M(D->G, k, i, a) * uv[i];
        w[a] = acc;
      }
      if (chol_rank1(L, n, w, pass ? -1.0 : 1.0)) return 2;
    }
  }
  /* C = L^-1 A' (:80-82), S = C'C, chol(S) (:83) */
  double* Cm = D->ALi;
  for (int r = 0; r < m; ++r) {
    double* col = Cm + (size_t)r * n;
    for (int a = 0; a < n; ++a) col[a] = M(D->A, m, r, a);
    for (int j = 0; j < n; ++j) {
      col[j] /= M(L, n, j, j);
      for (int i = j + 1; i < n; ++i) col[i] -= M(L, n, i, j) * col[j];
    }
  }
  for (int q = 0; q < m; ++q)
    for (int r = 0; r < m; ++r) {
      double acc = 0.0;
      for (int a = 0; a < n; ++a) acc += Cm[(size_t)r * n + a] * Cm[(size_t)q * n + a];
      M(D->S, m, r, q) = acc;
    }
  if (potrf_l(D->S, m)) return 3;
  return 0;
}

/* solve_kkt(::SparseSolver) (spsolver.jl:86-130) */
static void sqr_solve_kkt(dense_t* D, const cones_t* C, const scaling_t* S, const double* dx,
                          const double* dy, const double* dz, const double* ds, double* cx, double* cy,
                          double* cz, double* cs) {
  int n = D->n, m = D->m, k = D->k;
  iprod(C, D->k0, S->l, ds);
  scale_w(C, S, D->k0, D->k1);
  for (int i = 0; i < k; ++i) D->k2[i] = dz[i] - D->k1[i];
  iscale_w(C, S, D->k2, D->k1);
  iscale_w(C, S, D->k1, D->k1);
  for (int a = 0; a < n; ++a) {
    double acc = 0.0;
    for (int i = 0; i < k; ++i) acc += M(D->G, k, i, a) * D->k1[i];
    D->n0[a] = acc + dx[a];
  }
  if (D->sing)
    for (int a = 0; a < n; ++a) {
      double acc = 0.0;
      for (int r = 0; r < m; ++r) acc += M(D->A, m, r, a) * dy[r];
      D->n0[a] += acc;
    }
  for (int a = 0; a < n; ++a) D->n1[a] = D->n0[a];
  chol_solve_l(D->H, n, D->n1);
  for (int r = 0; r < m; ++r) {
    double acc = 0.0;
    for (int a = 0; a < n; ++a) acc += M(D->A, m, r, a) * D->n1[a];
    cy[r] = acc - dy[r];
  }
  chol_solve_l(D->S, m, cy);
  for (int r = 0; r < m; ++r) D->m0[r] = D->sing ? dy[r] - cy[r] : -cy[r];
  for (int a = 0; a < n; ++a) {
    double acc = 0.0;
    for (int r = 0; r < m; ++r) acc += M(D->A, m, r, a) * D->m0[r];
    D->n0[a] += acc;
  }
  for (int a = 0; a < n; ++a) cx[a] = D->n0[a];
  chol_solve_l(D->H, n, cx);
  for (int i = 0; i < k; ++i) {
    double acc = 0.0;
    for (int a = 0; a < n; ++a) acc += M(D->G, k, i, a) * cx[a];
    D->k1[i] = acc - D->k2[i];
  }
  iscale_w(C, S, D->k1, cz);
  iscale_w(C, S, cz, cz);
  scale_w(C, S, cz, D->k1);
  for (int i = 0; i < k; ++i) D->k0[i] -= D->k1[i];
  scale_w(C, S, D->k0, cs);
}

/* ---------------- workspace ---------------- */

typedef struct {
  scaling_t S;
  dense_t D;
  sqr_t Q;
  double *rd, *rp, *rz, *rs_, *dx, *dy, *dz, *ds, *rx, *ry, *rzz, *rss, *kt1, *kt2, *kt3, *nt1,
      *nt2, *mt1, *idel;
  double *K, *rhs; /* init system (n+m+k)^2 */
  int* piv;
  int n, m, k;
  void* block;
} ws_t;

static void* carve(char** p, size_t bytes) {
  void* r = *p;
  *p += (bytes + 63) & ~(size_t)63;
  return r;
}

static int ws_init(ws_t* w, int n, int m, int k, int ncones, int maxdim) {
  size_t N = (size_t)n + m + k;
  size_t need = 0;
#define SZ(x) need += (((x) + 63) & ~(size_t)63)
  SZ(3 * sizeof(double) * k * k);
  SZ(sizeof(double) * k * 2);
  SZ(sizeof(double) * ncones);
  SZ(sizeof(double) * maxdim * 2);
  SZ(sizeof(double) * n * n * 4);
  SZ(sizeof(double) * n * k);
  SZ(sizeof(double) * m * n);
  SZ(sizeof(double) * m * m);
  SZ(sizeof(double) * (3 * k + m + 2 * n));
  SZ(sizeof(double) * (size_t)20 * (n + m + k));
  SZ(sizeof(double) * N * N);
  SZ(sizeof(double) * N);
  SZ(sizeof(int) * N);
  SZ(sizeof(double) * 4 * k);
#undef SZ
  need += 64 * 64; /* per-carve alignment slack */
  char* p = (char*)calloc(1, need + 64);
  if (!p) return -1;
  w->block = p;
  w->n = n;
  w->m = m;
  w->k = k;
  w->S.k = k;
  w->S.W = carve(&p, sizeof(double) * k * k);
  w->S.iW = carve(&p, sizeof(double) * k * k);
  w->S.iWiW = carve(&p, sizeof(double) * k * k);
  w->S.l = carve(&p, sizeof(double) * k);
  w->S.wbs = carve(&p, sizeof(double) * k);
  w->S.mu = carve(&p, sizeof(double) * (ncones ? ncones : 1));
  w->S.sik = carve(&p, sizeof(double) * (maxdim ? maxdim : 1));
  w->S.zik = carve(&p, sizeof(double) * (maxdim ? maxdim : 1));
  w->D.n = n;
  w->D.m = m;
  w->D.k = k;
  w->D.structured = 0;
  w->D.cholsolve = 0;
  w->D.inv_yty = 0;
  w->D.C = NULL;
  w->D.AA = carve(&p, sizeof(double) * n * n);
  w->D.H = carve(&p, sizeof(double) * n * n);
  w->D.Li = carve(&p, sizeof(double) * n * n);
  w->D.Y = carve(&p, sizeof(double) * n * n);
  w->D.GWiWi = carve(&p, sizeof(double) * n * k);
  w->D.ALi = carve(&p, sizeof(double) * m * n);
  w->D.S = carve(&p, sizeof(double) * m * m);
  w->D.k0 = carve(&p, sizeof(double) * k);
  w->D.k1 = carve(&p, sizeof(double) * k);
  w->D.k2 = carve(&p, sizeof(double) * k);
  w->D.m0 = carve(&p, sizeof(double) * m);
  w->D.n0 = carve(&p, sizeof(double) * n);
  w->D.n1 = carve(&p, sizeof(double) * n);
  double** vecs[] = {&w->rd, &w->rp, &w->rz, &w->rs_, &w->dx, &w->dy, &w->dz,
                     &w->ds, &w->rx, &w->ry, &w->rzz, &w->rss, &w->kt1, &w->kt2,
                     &w->kt3, &w->nt1, &w->nt2, &w->mt1, &w->idel};
  for (size_t i = 0; i < sizeof(vecs) / sizeof(vecs[0]); ++i)
    *vecs[i] = carve(&p, sizeof(double) * (n + m + k));
  w->K = carve(&p, sizeof(double) * N * N);
  w->rhs = carve(&p, sizeof(double) * N);
  w->piv = carve(&p, sizeof(int) * N);
  w->Q.D = carve(&p, sizeof(double) * 4 * k);
  w->Q.iWd = w->Q.D + k;
  w->Q.u = w->Q.D + 2 * k;
  w->Q.v = w->Q.D + 3 * k;
  return 0;
}

static void ws_free(ws_t* w) { free(w->block); }

/* Dense LU with partial pivoting of the init system; returns 0 or 1 if singular. */
static int lu_solve(double* K, int N, double* b, int* piv) {
  for (int j = 0; j < N; ++j) {
    int p = j;
    double best = fabs(M(K, N, j, j));
    for (int i = j + 1; i < N; ++i)
      if (fabs(M(K, N, i, j)) > best) {
        best = fabs(M(K, N, i, j));
        p = i;
      }
    piv[j] = p;
    if (best == 0.0) return 1;
    if (p != j) {
      for (int q = 0; q < N; ++q) {
        double t = M(K, N, j, q);
        M(K, N, j, q) = M(K, N, p, q);
        M(K, N, p, q) = t;
      }
      double t = b[j];
      b[j] = b[p];
      b[p] = t;
    }
    double r = 1.0 / M(K, N, j, j);
    for (int i = j + 1; i < N; ++i) M(K, N, i, j) *= r;
    for (int q = j + 1; q < N; ++q) {
      double f = M(K, N, j, q);
      if (f != 0.0)
        for (int i = j + 1; i < N; ++i) M(K, N, i, q) -= M(K, N, i, j) * f;
    }
  }
  for (int i = 0; i < N; ++i) {
    double t = b[i];
    for (int q = 0; q < i; ++q) t -= M(K, N, i, q) * b[q];
    b[i] = t;
  }
  for (int i = N - 1; i >= 0; --i) {
    double t = b[i];
    for (int q = i + 1; q < N; ++q) t -= M(K, N, i, q) * b[q];
    b[i] = t / M(K, N, i, i);
  }
  return 0;
}

typedef struct {
  int32_t maxit;
  int32_t sigma_exp;
  double tol;
  double step;
  double init_eps;
  int32_t flags;
  int32_t reserved;
} params_t; /* mirrors socp_params */

#define F_WARM 2
#define OR_F_STRUCTURED 16 /* oracle-only: the build's structured algorithm (CPU baseline) */
#define OR_F_SQR 32        /* oracle-only: SqrScaling + SparseSolver (spsolver.jl) instead of DenseSolver */
#define OR_F_CHOLSOLVE 64  /* oracle-only, with OR_F_STRUCTURED: triangular solves instead of the explicit Li */
#define OR_F_INV_YTY 128   /* oracle-only, with OR_F_STRUCTURED: Li = Y'Y, Y = L^-1 (the kernels' explicit inverse) */

static double dot(const double* a, const double* b, int n) {
  double s = 0.0;
  for (int i = 0; i < n; ++i) s += a[i] * b[i];
  return s;
}
static double nrm2(const double* a, int n) { return sqrt(dot(a, a, n)); }

static double powi_sig(double x, int e) {
  if (e == 3) return x * x * x; /* Julia literal_pow: x*x*x */
  return pow(x, (double)e);
}

/* Initial point (solver.jl:68-104): exact solve of [0 A' G'; A 0 0; G 0 -I], then shift. */
static int init_point(ws_t* w, const cones_t* C, const double* c, const double* A, const double* b,
                      const double* G, const double* h, const params_t* P, double* x, double* y,
                      double* z, double* s) {
  int n = w->n, m = w->m, k = w->k, N = n + m + k;
  memset(w->K, 0, sizeof(double) * (size_t)N * N);
  for (int j = 0; j < n; ++j) {
    for (int i = 0; i < m; ++i) {
      M(w->K, N, n + i, j) = M(A, m, i, j);
      M(w->K, N, j, n + i) = M(A, m, i, j);
    }
    for (int i = 0; i < k; ++i) {
      M(w->K, N, n + m + i, j) = M(G, k, i, j);
      M(w->K, N, j, n + m + i) = M(G, k, i, j);
    }
  }
  for (int i = 0; i < k; ++i) M(w->K, N, n + m + i, n + m + i) = -1.0;
  for (int j = 0; j < n; ++j) w->rhs[j] = -c[j];
  for (int i = 0; i < m; ++i) w->rhs[n + i] = b[i];
  for (int i = 0; i < k; ++i) w->rhs[n + m + i] = h[i];
  if (lu_solve(w->K, N, w->rhs, w->piv)) return 2;
  make_e(C, w->idel);
  const double* iz = w->rhs + n + m;
  double* miz = w->kt1;
  for (int i = 0; i < k; ++i) miz[i] = -iz[i];
  double alphp = max_step(C, miz);
  double alphd = max_step(C, iz);
  for (int i = 0; i < k; ++i)
    s[i] = (fabs(alphp) < P->init_eps) ? -iz[i] : -iz[i] + (1.0 + alphp) * w->idel[i];
  for (int i = 0; i < k; ++i)
    z[i] = (fabs(alphd) < P->init_eps) ? iz[i] : iz[i] + (1.0 + alphd) * w->idel[i];
  for (int j = 0; j < n; ++j) x[j] = w->rhs[j];
  for (int i = 0; i < m; ++i) y[i] = w->rhs[n + i];
  return 0;
}

/* One problem: solve_socp (solver.jl:40-153).  trace (optional): iterates at
 * the start of every iteration, trace[t*(n+m+2k) + ...] = (x,y,z,s). */
static void solve_one(ws_t* w, const cones_t* C, const double* c, const double* A,
                      const double* b, const double* G, const double* h, int sing,
                      const params_t* P, double* x, double* y, double* z, double* s, int* iters_out,
                      int* status_out, double* res, double* trace, int max_trace) {
  int n = w->n, m = w->m, k = w->k;
  scaling_t* S = &w->S;
  dense_t* D = &w->D;
  D->A = A;
  D->G = G;
  D->sing = sing;
  D->C = C;
  D->structured = (P->flags & OR_F_STRUCTURED) != 0;
  D->cholsolve = D->structured && (P->flags & OR_F_CHOLSOLVE) != 0;
  D->inv_yty = D->structured && !D->cholsolve && (P->flags & OR_F_INV_YTY) != 0;
  const int sqr = (P->flags & OR_F_SQR) != 0;
#define KKT(a, b_, c_, d, e, f, g, h_) \
  (sqr ? sqr_solve_kkt(D, C, S, a, b_, c_, d, e, f, g, h_) : solve_kkt(D, C, S, a, b_, c_, d, e, f, g, h_))
  /* DenseSolver ctor: AA = A'A (densesolver.jl:31-32) */
  for (int bq = 0; bq < n; ++bq)
    for (int a = 0; a < n; ++a) {
      double acc = 0.0;
      for (int r = 0; r < m; ++r) acc += M(A, m, r, a) * M(A, m, r, bq);
      M(D->AA, n, a, bq) = acc;
    }
  memset(S->W, 0, sizeof(double) * (size_t)k * k);
  memset(S->iW, 0, sizeof(double) * (size_t)k * k);
  int status = 1, iters = 0;
  make_e(C, w->idel);
  if (!(P->flags & F_WARM)) {
    if (init_point(w, C, c, A, b, G, h, P, x, y, z, s)) {
      status = 2;
      goto done;
    }
  }
  int dg = deg(C);
  int stride = n + m + 2 * k;
  for (int it = 0; it < P->maxit; ++it) {
    if (trace && it < max_trace) {
      double* t = trace + (size_t)it * stride;
      memcpy(t, x, sizeof(double) * n);
      memcpy(t + n, y, sizeof(double) * m);
      memcpy(t + n + m, z, sizeof(double) * k);
      memcpy(t + n + m + k, s, sizeof(double) * k);
    }
    int dom = 0;
    if (sqr)
      sqr_compute_scaling(C, S, &w->Q, s, z, &dom);
    else
      compute_scaling_x(C, S, s, z, &dom, D->structured);
    if (dom) {
      status = 4;
      break;
    }
    const double* l = S->l;
    for (int j = 0; j < n; ++j) {
      double a1 = 0.0, a2 = 0.0;
      for (int i = 0; i < m; ++i) a1 += M(A, m, i, j) * y[i];
      for (int i = 0; i < k; ++i) a2 += M(G, k, i, j) * z[i];
      w->nt1[j] = a1;
      w->nt2[j] = a2;
    }
    for (int j = 0; j < n; ++j) w->dx[j] = w->nt1[j] + w->nt2[j] + c[j];
    for (int i = 0; i < m; ++i) w->mt1[i] = 0.0;
    for (int i = 0; i < k; ++i) w->kt1[i] = 0.0;
    for (int j = 0; j < n; ++j) {
      for (int i = 0; i < m; ++i) w->mt1[i] += M(A, m, i, j) * x[j];
      for (int i = 0; i < k; ++i) w->kt1[i] += M(G, k, i, j) * x[j];
    }
    for (int i = 0; i < m; ++i) w->dy[i] = w->mt1[i] - b[i];
    for (int i = 0; i < k; ++i) w->dz[i] = w->kt1[i] + s[i] - h[i];
    vprod(C, w->ds, l, l);
    if (nrm2(w->dx, n) + nrm2(w->dy, m) + dot(z, s, k) < P->tol) {
      status = 0;
      break;
    }
    for (int j = 0; j < n; ++j) w->dx[j] *= -1.0;
    for (int i = 0; i < m; ++i) w->dy[i] *= -1.0;
    for (int i = 0; i < k; ++i) w->dz[i] *= -1.0;
    for (int i = 0; i < k; ++i) w->ds[i] *= -1.0;
    int st = sqr ? sqr_setup_iter(D, C, &w->Q) : setup_iter(D, S);
    if (st) {
      status = st;
      break;
    }
    KKT(w->dx, w->dy, w->dz, w->ds, w->rx, w->ry, w->rzz, w->rss);
    scale_w(C, S, w->rzz, w->kt3);
    iscale_w(C, S, w->rss, w->kt2);
    double t = compute_step(C, l, w->kt3, w->kt2, &dom);
    if (dom) {
      status = 4;
      break;
    }
    double ll = dot(l, l, k);
    double rho = 1.0 - t - t * t * dot(w->kt2, w->kt3, k) / ll;
    double sig = powi_sig(jmax(0.0, jmin(1.0, rho)), P->sigma_exp);
    double mu = ll / dg;
    double scfact = 1.0 - sig;
    vprod(C, w->kt1, w->kt2, w->kt3);
    for (int i = 0; i < k; ++i) w->kt2[i] = sig * mu * w->idel[i];
    for (int i = 0; i < k; ++i) w->ds[i] += w->kt2[i] - w->kt1[i];
    for (int j = 0; j < n; ++j) w->dx[j] *= scfact;
    for (int i = 0; i < m; ++i) w->dy[i] *= scfact;
    for (int i = 0; i < k; ++i) w->dz[i] *= scfact;
    KKT(w->dx, w->dy, w->dz, w->ds, w->rx, w->ry, w->rzz, w->rss);
    scale_w(C, S, w->rzz, w->kt3);
    iscale_w(C, S, w->rss, w->kt2);
    double step = compute_step(C, l, w->kt3, w->kt2, &dom);
    if (dom) {
      status = 4;
      break;
    }
    step *= P->step;
    for (int j = 0; j < n; ++j) x[j] += w->rx[j] * step;
    for (int i = 0; i < m; ++i) y[i] += w->ry[i] * step;
    for (int i = 0; i < k; ++i) z[i] += w->rzz[i] * step;
    for (int i = 0; i < k; ++i) s[i] += w->rss[i] * step;
    iters = it + 1;
  }
done:
  if (res) {
    for (int j = 0; j < n; ++j) {
      double a1 = 0.0, a2 = 0.0;
      for (int i = 0; i < m; ++i) a1 += M(A, m, i, j) * y[i];
      for (int i = 0; i < k; ++i) a2 += M(G, k, i, j) * z[i];
      w->dx[j] = a1 + a2 + c[j];
    }
    for (int i = 0; i < m; ++i) {
      double acc = 0.0;
      for (int j = 0; j < n; ++j) acc += M(A, m, i, j) * x[j];
      w->dy[i] = acc - b[i];
    }
    res[0] = nrm2(w->dx, n);
    res[1] = nrm2(w->dy, m);
    res[2] = dot(z, s, k);
  }
  *iters_out = iters;
  *status_out = status;
#undef KKT
}

static int max_dim(const cones_t* C) {
  int md = 1;
  for (int c = 0; c < C->ncones; ++c)
    if (C->dim[c] > md) md = C->dim[c];
  return md;
}

/* ================= exported API (ctypes) ================= */

EXPORT void or_make_e(int nc, const int32_t* kind, const int32_t* offs, const int32_t* dim,
                      double* r) {
  cones_t C = {nc, kind, offs, dim};
  make_e(&C, r);
}
EXPORT void or_vprod(int nc, const int32_t* kind, const int32_t* offs, const int32_t* dim,
                     double* t, const double* u, const double* v) {
  cones_t C = {nc, kind, offs, dim};
  vprod(&C, t, u, v);
}
EXPORT void or_iprod(int nc, const int32_t* kind, const int32_t* offs, const int32_t* dim,
                     double* t, const double* lam, const double* v) {
  cones_t C = {nc, kind, offs, dim};
  iprod(&C, t, lam, v);
}
EXPORT int or_cgt(int nc, const int32_t* kind, const int32_t* offs, const int32_t* dim,
                  const double* x, const double* dx) {
  cones_t C = {nc, kind, offs, dim};
  return cgt(&C, x, dx);
}
EXPORT int or_deg(int nc, const int32_t* kind, const int32_t* offs, const int32_t* dim) {
  cones_t C = {nc, kind, offs, dim};
  return deg(&C);
}
EXPORT double or_max_step(int nc, const int32_t* kind, const int32_t* offs, const int32_t* dim,
                          const double* x) {
  cones_t C = {nc, kind, offs, dim};
  return max_step(&C, x);
}
EXPORT double or_compute_step(int nc, const int32_t* kind, const int32_t* offs,
                              const int32_t* dim, const double* l, const double* ds,
                              const double* dz, int* dom) {
  cones_t C = {nc, kind, offs, dim};
  *dom = 0;
  return compute_step(&C, l, ds, dz, dom);
}

/* compute_scaling for one (s,z): outputs W, iW, iWiW (k x k col-major), l, mu, wbs. */
EXPORT int or_compute_scaling(int nc, const int32_t* kind, const int32_t* offs,
                              const int32_t* dim, int k, const double* s, const double* z,
                              double* W, double* iW, double* iWiW, double* l, double* mu,
                              double* wbs) {
  cones_t C = {nc, kind, offs, dim};
  int md = max_dim(&C);
  double* tmp = (double*)malloc(sizeof(double) * 2 * md);
  scaling_t S = {k, W, iW, iWiW, l, mu, wbs, tmp, tmp + md};
  memset(W, 0, sizeof(double) * (size_t)k * k);
  memset(iW, 0, sizeof(double) * (size_t)k * k);
  int dom = 0;
  compute_scaling(&C, &S, s, z, &dom);
  free(tmp);
  return dom ? 4 : 0;
}

EXPORT void or_scale(int nc, const int32_t* kind, const int32_t* offs, const int32_t* dim,
                     const double* wbs, const double* mu, const double* x, double* out, int inv) {
  cones_t C = {nc, kind, offs, dim};
  scaling_t S;
  memset(&S, 0, sizeof(S));
  S.wbs = (double*)wbs;
  S.mu = (double*)mu;
  if (inv)
    iscale_w(&C, &S, x, out);
  else
    scale_w(&C, &S, x, out);
}

/* compute_scaling + setup_iter + solve_kkt for one problem at iterate (s,z).
 * Optional outputs: H (n x n, the matrix before factorisation), Li. Returns status. */
EXPORT int or_kkt_single(int nc, const int32_t* kind, const int32_t* offs, const int32_t* dim,
                         int n, int m, int k, const double* A, const double* G, int sing,
                         const double* s, const double* z, const double* dx, const double* dy,
                         const double* dz, const double* ds, double* cx, double* cy, double* cz,
                         double* cs, double* Hout, double* Liout, int structured) {
  cones_t C = {nc, kind, offs, dim};
  ws_t w;
  if (ws_init(&w, n, m, k, nc, max_dim(&C))) return -1;
  w.D.A = A;
  w.D.G = G;
  w.D.sing = sing;
  w.D.C = &C;
  w.D.structured = structured != 0; /* the kernels' order (F_STRUCTURED); H output: reference order only */
  w.D.cholsolve = (structured & 2) != 0; /* 2 | 1: with the triangular solves (OR_F_CHOLSOLVE) */
  w.D.inv_yty = (structured & 1) && !(structured & 2) && (structured & 4); /* 4 | 1: Li = Y'Y (OR_F_INV_YTY) */
  if (structured) Hout = NULL;
  if (structured & 2) Liout = NULL;
  for (int bq = 0; bq < n; ++bq)
    for (int a = 0; a < n; ++a) {
      double acc = 0.0;
      for (int r = 0; r < m; ++r) acc += M(A, m, r, a) * M(A, m, r, bq);
      M(w.D.AA, n, a, bq) = acc;
    }
  int dom = 0;
  compute_scaling_x(&C, &w.S, s, z, &dom, structured);
  int st = 0;
  if (dom) {
    st = 4;
  } else {
    /* H before the factorisation overwrites it */
    int nn = n;
    st = setup_iter(&w.D, &w.S);
    if (Hout) {
      for (int bq = 0; bq < nn; ++bq)
        for (int a = 0; a < nn; ++a) {
          double acc = 0.0;
          for (int i = 0; i < k; ++i) acc += M(w.D.GWiWi, nn, a, i) * M(G, k, i, bq);
          M(Hout, nn, a, bq) = acc + (sing ? M(w.D.AA, nn, a, bq) : 0.0);
        }
    }
    if (!st) {
      solve_kkt(&w.D, &C, &w.S, dx, dy, dz, ds, cx, cy, cz, cs);
      if (Liout) memcpy(Liout, w.D.Li, sizeof(double) * (size_t)n * n);
    }
  }
  ws_free(&w);
  return st;
}

/* SqrScaling + setup_iter(::SparseSolver) + solve_kkt for one problem at (s,z)
 * (the runtests.jl:95-128 sequence).  Optional outputs: Lout (n x n, the
 * factor of H after modify_factors!), l/wbs (k), mu (nc).  Returns status. */
EXPORT int or_sqr_kkt_single(int nc, const int32_t* kind, const int32_t* offs, const int32_t* dim,
                             int n, int m, int k, const double* A, const double* G, int sing,
                             const double* s, const double* z, const double* dx, const double* dy,
                             const double* dz, const double* ds, double* cx, double* cy, double* cz,
                             double* cs, double* Lout, double* lout, double* wbsout, double* muout) {
  cones_t C = {nc, kind, offs, dim};
  ws_t w;
  if (ws_init(&w, n, m, k, nc, max_dim(&C))) return -1;
  w.D.A = A;
  w.D.G = G;
  w.D.sing = sing;
  w.D.C = &C;
  for (int bq = 0; bq < n; ++bq)
    for (int a = 0; a < n; ++a) {
      double acc = 0.0;
      for (int r = 0; r < m; ++r) acc += M(A, m, r, a) * M(A, m, r, bq);
      M(w.D.AA, n, a, bq) = acc;
    }
  int dom = 0;
  sqr_compute_scaling(&C, &w.S, &w.Q, s, z, &dom);
  if (lout) memcpy(lout, w.S.l, sizeof(double) * k);
  if (wbsout) memcpy(wbsout, w.S.wbs, sizeof(double) * k);
  if (muout) memcpy(muout, w.S.mu, sizeof(double) * nc);
  int st = dom ? 4 : sqr_setup_iter(&w.D, &C, &w.Q);
  if (!st) {
    sqr_solve_kkt(&w.D, &C, &w.S, dx, dy, dz, ds, cx, cy, cz, cs);
    if (Lout) memcpy(Lout, w.D.H, sizeof(double) * (size_t)n * n);
  }
  ws_free(&w);
  return st;
}

/* Batched solve (one problem per OpenMP thread, static schedule).  Layout as
 * include/socp.h.  res may be NULL (else 3 per problem). Returns 0 / -1. */
EXPORT int or_batch_solve(int64_t B, int n, int m, int k, int nc, const int32_t* kind,
                          const int32_t* offs, const int32_t* dim, const double* c,
                          const double* A, const double* b, const double* G, const double* h,
                          const uint8_t* sing, const params_t* P, double* x, double* y, double* z,
                          double* s, int32_t* iters, int32_t* status, double* res, int nthreads) {
  cones_t C = {nc, kind, offs, dim};
  int md = max_dim(&C);
  int err = 0;
#ifdef _OPENMP
  if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads)
#endif
  {
    ws_t w;
    if (ws_init(&w, n, m, k, nc, md)) {
#ifdef _OPENMP
#pragma omp atomic write
#endif
      err = -1;
    } else {
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
      for (int64_t p = 0; p < B; ++p) {
        int it, st;
        solve_one(&w, &C, c + p * n, A + p * (int64_t)m * n, b + p * m, G + p * (int64_t)k * n,
                  h + p * k, sing ? sing[p] : 0, P, x + p * n, y + p * m, z + p * k, s + p * k,
                  &it, &st, res ? res + 3 * p : NULL, NULL, 0);
        iters[p] = it;
        status[p] = st;
      }
      ws_free(&w);
    }
  }
  return err;
}

/* Single problem with a per-iteration trace of (x,y,z,s); trace has room for
 * max_trace iterates of n+m+2k doubles. */
EXPORT int or_solve_trace(int n, int m, int k, int nc, const int32_t* kind, const int32_t* offs,
                          const int32_t* dim, const double* c, const double* A, const double* b,
                          const double* G, const double* h, int sing, const params_t* P,
                          double* x, double* y, double* z, double* s, int32_t* iters,
                          int32_t* status, double* res, double* trace, int max_trace) {
  cones_t C = {nc, kind, offs, dim};
  ws_t w;
  if (ws_init(&w, n, m, k, nc, max_dim(&C))) return -1;
  int it, st;
  solve_one(&w, &C, c, A, b, G, h, sing, P, x, y, z, s, &it, &st, res, trace, max_trace);
  *iters = it;
  *status = st;
  ws_free(&w);
  return 0;
}

/* Initial point only (solver.jl:68-104). */
EXPORT int or_init_point(int n, int m, int k, int nc, const int32_t* kind, const int32_t* offs,
                         const int32_t* dim, const double* c, const double* A, const double* b,
                         const double* G, const double* h, const params_t* P, double* x, double* y,
                         double* z, double* s) {
  cones_t C = {nc, kind, offs, dim};
  ws_t w;
  if (ws_init(&w, n, m, k, nc, max_dim(&C))) return -1;
  int st = init_point(&w, &C, c, A, b, G, h, P, x, y, z, s);
  ws_free(&w);
  return st;
}

/* `sing` rule of Problem (Socp.jl:49-56): 1 if cholesky(G'G) fails. */
EXPORT int or_sing(int n, int k, const double* G) {
  double* H = (double*)malloc(sizeof(double) * (size_t)n * n);
  for (int bq = 0; bq < n; ++bq)
    for (int a = 0; a < n; ++a) {
      double acc = 0.0;
      for (int i = 0; i < k; ++i) acc += M(G, k, i, a) * M(G, k, i, bq);
      M(H, n, a, bq) = acc;
    }
  int f = potrf_u(H, n) != 0;
  free(H);
  return f;
}

/* ---------------- generator restatement ---------------- */

static inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
static inline double gen_u(uint64_t seed, uint64_t p, uint64_t e) {
  uint64_t u = splitmix64(seed ^ ((p << 24) | e));
  return (double)(u >> 11) * 0x1.0p-53;
}

/* CPU restatement of socp_generate; must be built with -ffp-contract=off. */
EXPORT void or_generate(int64_t B, int n, int m, int k, int nc, const int32_t* kind,
                        const int32_t* offs, const int32_t* dim, uint64_t seed,
                        int64_t first_problem, double* c, double* A, double* b, double* G,
                        double* h) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
  for (int64_t p = 0; p < B; ++p) {
    uint64_t gp = (uint64_t)(first_problem + p);
    double* Gp = G + p * (int64_t)k * n;
    double* Ap = A + p * (int64_t)m * n;
    double* x0 = (double*)malloc(sizeof(double) * (n + m + 2 * k));
    double* y0 = x0 + n;
    double* s0 = y0 + m;
    double* z0 = s0 + k;
    uint64_t e = 0;
    for (int64_t q = 0; q < (int64_t)k * n; ++q) Gp[q] = 2.0 * gen_u(seed, gp, e++) - 1.0;
    for (int64_t q = 0; q < (int64_t)m * n; ++q) Ap[q] = 2.0 * gen_u(seed, gp, e++) - 1.0;
    for (int j = 0; j < n; ++j) x0[j] = 2.0 * gen_u(seed, gp, e++) - 1.0;
    for (int i = 0; i < m; ++i) y0[i] = 2.0 * gen_u(seed, gp, e++) - 1.0;
    for (int cc = 0; cc < nc; ++cc) {
      int o = offs[cc], d = dim[cc];
      for (int which = 0; which < 2; ++which) {
        double* v = which ? z0 : s0;
        if (kind[cc] == POC) {
          for (int i = 0; i < d; ++i) v[o + i] = 0.5 + gen_u(seed, gp, e++);
        } else {
          double sq = 0.0;
          for (int i = 1; i < d; ++i) {
            double t = 2.0 * gen_u(seed, gp, e++) - 1.0;
            v[o + i] = t;
            sq += t * t;
          }
          v[o] = sqrt(sq) + 0.5 + gen_u(seed, gp, e++);
        }
      }
    }
    for (int i = 0; i < k; ++i) {
      double acc = 0.0;
      for (int j = 0; j < n; ++j) acc += M(Gp, k, i, j) * x0[j];
      h[p * k + i] = acc + s0[i];
    }
    for (int i = 0; i < m; ++i) {
      double acc = 0.0;
      for (int j = 0; j < n; ++j) acc += M(Ap, m, i, j) * x0[j];
      b[p * m + i] = acc;
    }
    for (int j = 0; j < n; ++j) {
      double t = 0.0, u = 0.0;
      for (int i = 0; i < m; ++i) t += M(Ap, m, i, j) * y0[i];
      for (int i = 0; i < k; ++i) u += M(Gp, k, i, j) * z0[i];
      c[p * n + j] = -(t + u);
    }
    free(x0);
  }
}
