// socp_large.hip — the blocked batched dense SOCP IPM kernel (gfx950) for the
// shapes beyond the register-resident kernel: n and m up to 512, k as LDS
// allows.  BASELINE config C4 (n=512, m=64, k=640, 8 SOC(80) cones) runs here.
//
// One 512-thread workgroup (8 wavefronts) owns one problem for its whole solve;
// persistent workgroups pull problem indices from an atomic counter.  The
// problem's vectors live in LDS (C4: 126 KiB), its matrices in the workgroup's
// slot of an HBM workspace, all column-major:
//   Xw = W^-1 G (KP x NPAD), rebuilt from G at every factorisation;
//   Hm = H -> -H^-1 (sweep, lower triangle) -> Li = H^-1 (both triangles);
//   Ap, At = A zero-padded, column- and row-major;  Tm = Li A' (NPAD x MPAD);
//   Sm = S -> S^-1;  Yp = the sweep's captured pivot rows (64 x max(NPAD, MPAD)).
// Per iteration (solver.jl:105-151) the algebra of the register kernel:
//   H = X'X (+A'A) as f64-MFMA 64x64 blocks: the reference's iWiW GEMM and
//     G'*iWiW*G products (scalings.jl:108, densesolver.jl:42-46) structurally;
//   Li = H^-1 by a blocked symmetric Gauss-Jordan sweep (densesolver.jl:47-48):
//     each 64-pivot row panel is swept in registers (a thread holds 8 panel
//     rows x NPAD/64 columns; the pivots are the Cholesky pivots, so the
//     positive-definiteness test is cholesky!'s), and the rank-64 update of
//     the other blocks is deferred into one MFMA Gram product per panel;
//   T = Li A', S = A T and S^-1 by the same sweep (densesolver.jl:49-51);
//   the two KKT solves (densesolver.jl:54-90) as mat-vecs over the workspace.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#ifndef SOCP_LG_TILE_INPLACE
#define SOCP_LG_TILE_INPLACE 1  // factor_tile's trailing updates in place (0: copying form, A/B)
#endif
#define SOCP_MULTI_WAVE 1  // LANE_IDS / factor_tile: lanes of 8-wavefront workgroups
#include "socp_kernels.hpp"

// Tuning builds only (never the product): SOCP_LREP bit b runs an idempotent
// phase of the blocked kernel twice, so that the time and the PMC traffic of
// one instance are the build's difference to the product -- 1 X = W^-1 G,
// 2 the SYRK, 4 the solves' G'v, 8 their G v, 16 their triangular solves,
// 32 Z = L^-1 A' and S = Z'Z, 64 the residuals' G pass, 128 compute_scaling,
// 256 the solves' head (iprod / scale / k2 / W^-1 W^-1)
#ifndef SOCP_LREP
#define SOCP_LREP 0
#endif
#define LREP(b) ((SOCP_LREP & (b)) ? 2 : 1)
#ifndef SOCP_LG_CATCH_SPLIT
#define SOCP_LG_CATCH_SPLIT 1  // chol_nb: split the last panels' catch-up blocks by 16-column groups
#endif
#ifndef SOCP_LG_SYRK_SYNC
#define SOCP_LG_SYRK_SYNC 128  // form_H: rows of k between workgroup barriers (0: none)
#endif
#ifndef SOCP_LG_FX_RS
#define SOCP_LG_FX_RS 1  // W^-1 G: the 32 cone sums of a pass by one reduce-scatter (0: 32 all-reduces)
#endif
#ifndef SOCP_LG_KO
#define SOCP_LG_KO 0  // timing knock-outs of the W^-1 G phase (tuning builds only; results wrong)
#endif
#ifndef SOCP_LG_SYRK_ORDER
#define SOCP_LG_SYRK_ORDER 1  // form_H with SYRK_SYNC at NPAD = 512: the panel-sharing round order (0: row-major)
#endif
#ifndef SOCP_LG_SYRK_UNROLL
#define SOCP_LG_SYRK_UNROLL 1  // blk_gemm's k loop (16 rows per step)
#endif
#ifndef SOCP_LG_GRAM_UNROLL
#define SOCP_LG_GRAM_UNROLL 1  // gram_blkT's 16-row steps per unrolled round
#endif
#ifndef SOCP_LG_CATCH_SPLIT_K
#define SOCP_LG_CATCH_SPLIT_K 2  // split when at most NW / K blocks are left
#endif
#ifndef SOCP_LG_ZU
#define SOCP_LG_ZU 8  // Z = L^-1 A' update: 4-row k-steps per batch of loads (P0 is a multiple of 64; 16: the same time)
#endif

namespace socp {
namespace lg {

constexpr int NW = 8;              // wavefronts per workgroup
constexpr int NTH = 64 * NW;       // threads per workgroup
constexpr int NBT = LARGE_NB_MAX;  // 64-column blocks a swept panel row may span
constexpr int CG = 8;              // columns per wavefront pass in the G' / W^-1 G passes
constexpr int NOPAD = 1 << 30;     // store_blk: no identity padding

// Workspace and problem pointers in the global address space (otherwise, once
// they pass through the stack object of an out-of-line member call, the
// compiler sees generic pointers and emits flat instructions).
typedef __attribute__((address_space(1))) double gdbl;
typedef __attribute__((address_space(1))) const double gcdbl;
typedef double dbl2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(1))) const dbl2 gcdbl2;

extern __shared__ double lg_lds[];
// The problem's vectors: in LDS, or (GV: shapes whose vectors exceed the
// 160 KiB of a CU's LDS, e.g. k = 1000 at n = 512) in the workgroup's slot of
// the HBM workspace -- Large::lvref picks at compile time.
#define LV(i) lvref(i)
// Workgroup barrier.  Global stores read by other wavefronts after it (the
// workspace) are drained first; all waves of the workgroup share the CU's L1.
#define BAR()                                       \
  do {                                              \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); \
    __syncthreads();                                \
  } while (0)
// LDS-only barrier: the global stores in flight stay in flight (a
// __syncthreads would drain them first, one store round trip per barrier)
#define LDS_BAR()                                                     \
  do {                                                                \
    if constexpr (GV) {                                               \
      BAR(); /* the vectors are global memory: drain the stores too */ \
    } else {                                                          \
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");    \
    }                                                                 \
  } while (0)

// Diagnostic build (-DSOCP_DIAG): thread 0 adds per-phase s_memtime deltas
// into u64 totals at LDS o_red + 16 (its own timeline: the phases end in
// workgroup barriers), flushed to args.stamps once per workgroup.
#ifdef SOCP_DIAG
#define LSTAMP(i)                                                                          \
  do {                                                                                     \
    if (!GV && tid == 0) {                                                                 \
      const uint64_t t_ = __builtin_amdgcn_s_memtime();                                    \
      reinterpret_cast<unsigned long long*>(lg_lds + L.o_red + 16)[(i)] += t_ - st_last;    \
      st_last = t_;                                                                        \
    }                                                                                      \
  } while (0)
#else
#define LSTAMP(i) \
  do {            \
  } while (0)
#endif

// wave-uniform sum / max: DPP inclusive scan to lane 63, broadcast by readlane
__device__ __forceinline__ double wave_sum(double v) {
  double x[1] = {v};
  dpp_scan<1>(x, (int)(threadIdx.x & 63), 0, false);
  return readlane_d(x[0], 63);
}
// sum over each 16-lane row (every lane of the row gets it): DPP rotations
__device__ __forceinline__ double row16_sum(double v) {
  v += dpp_all<0x128>(v);  // row_ror:8
  v += dpp_all<0x124>(v);  // row_ror:4
  v += dpp_all<0x122>(v);  // row_ror:2
  v += dpp_all<0x121>(v);  // row_ror:1
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
  double x[1] = {v};
  dpp_scan<1>(x, (int)(threadIdx.x & 63), 0, true);
  return readlane_d(x[0], 63);
}

#ifndef SOCP_LG_PANEL
#define SOCP_LG_PANEL 1  // 0: the per-pivot rank-1 sweep of a panel (A/B builds)
#endif
#ifndef SOCP_LG_INV_CHOL
#define SOCP_LG_INV_CHOL 1  // 0: explicit inverses by the Gauss-Jordan sweep (A/B builds)
#endif
#ifndef SOCP_LG_CHOL
#define SOCP_LG_CHOL 1  // 0: Li = H^-1 formed (A/B builds)
#endif

// C += U'V (NEG = 1: C -= U'V) for C/D-layout 16x16 tiles (socp_small.hpp's
// tile algebra: lane (g, cl) holds X[g+4r][cl] in register r)
template <int NEG>
__device__ __forceinline__ d4 tile_mm(const d4& U, const d4& V, d4 C) {
#pragma unroll
  for (int s = 0; s < 4; ++s) C = __builtin_amdgcn_mfma_f64_16x16x4f64(U[s], V[s], C, 0, 0, NEG);
  return C;
}

// XI (SOCP_F_EXPLICIT_INVERSE): Li = H^-1 formed from the Cholesky factor
// (chol_inverse), the reference's operation order (densesolver.jl:47-48),
// instead of the triangular solves against H = L L'.
// GV: the vectors in global memory (LV above).
template <bool XI, bool GV>
struct Large {
  static constexpr bool CHOL = SOCP_LG_CHOL && !XI;
  // where Li = H^-1 is formed (XI, and every shape of a SOCP_LG_CHOL=0 build):
  // from the Cholesky factor, Li = L^-T L^-1 (chol_inverse), as
  // densesolver.jl:47-48 forms it; S^-1 likewise (0: the Gauss-Jordan sweep)
  static constexpr bool INV_CHOL = SOCP_LG_INV_CHOL && !CHOL;
  gdbl* gvec = nullptr;  // GV: this workgroup's vector region (workspace slot)
  __device__ __forceinline__ auto& lvref(int i) const {
    if constexpr (GV)
      return gvec[i];
    else
      return lg_lds[i];
  }
  const SmallArgs& a;
  const LargeLayout L;
  const int n, m, k, nc, tid, lane, wv;
  int kpoc, csoc;  // POC elements (POC cones come first) and index of the first SOC cone
  bool sing;
  gcdbl* Gp;
  gdbl *Xw, *Hm, *Ap, *At, *Yp, *Rv, *Tm, *Sm, *Vr;
  gdbl* const ws0;
  gdbl* const rec0;
  const int64_t wstride;
  // LDS vector offsets (doubles)
  int H_, Z_, S_, DZ, DS, RZ, RS, LAM, WB, CA, K0, K1, K2, T1, T2;
  int C_, X_, RD, RX, N0, TN;
  int B_, Y_, RP, RY, M0;
  uint64_t st_last = 0;

  __device__ Large(const LargeArgs& la)
      : a(la.a), L(large_layout(la.a.n, la.a.m, la.a.k)), n(la.a.n), m(la.a.m), k(la.a.k),
        nc(la.a.nc), tid(threadIdx.x), lane(threadIdx.x & 63),
        wv(__builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6)), ws0((gdbl*)la.ws), rec0((gdbl*)la.rec),
        wstride(la.wstride) {
    set_slot(blockIdx.x);
    const int kl = L.o_kvl, kd = L.o_kvd, KP = L.KP;
    H_ = kl;
    Z_ = kl + KP;
    S_ = kl + 2 * KP;
    DZ = kl + 3 * KP;
    DS = kl + 4 * KP;
    LAM = kl + 5 * KP;
    WB = kl + 6 * KP;
    CA = kl + 7 * KP;
    // dead while a factorisation runs (under the staged SYRK's buffers)
    RZ = kd;
    RS = kd + KP;
    K0 = kd + 2 * KP;
    K1 = kd + 3 * KP;
    K2 = kd + 4 * KP;
    T1 = kd + 5 * KP;
    T2 = kd + 6 * KP;
    const int nv = L.o_nv, NP = L.NPAD;
    C_ = nv;
    X_ = nv + NP;
    RD = nv + 2 * NP;
    RX = nv + 3 * NP;
    N0 = nv + 4 * NP;
    TN = nv + 5 * NP;
    const int mv = L.o_mv, MP = L.MPAD;
    B_ = mv;
    Y_ = mv + MP;
    RP = mv + 2 * MP;
    RY = mv + 3 * MP;
    M0 = mv + 4 * MP;
    kpoc = 0;
    csoc = 0;
    for (int c = 0; c < nc && a.cones.kind[c] == POC_K; ++c) {
      kpoc += a.cones.dim[c];
      csoc = c + 1;
    }
    sing = false;
    Gp = (gcdbl*)a.G;
  }

  __device__ void set_slot(int64_t slot) {
    gdbl* ws = ws0 + slot * wstride;
    Xw = ws + L.w_x;
    Hm = ws + L.w_h;
    Ap = ws + L.w_ap;
    At = ws + L.w_at;
    Yp = ws + L.w_yp;
    Rv = ws + L.w_rv;
    Tm = ws + L.w_t;
    Sm = ws + L.w_s;
    Vr = ws + L.w_v;
    if constexpr (GV) gvec = ws + L.w_lv;
  }
  // the matrices solve_kkt reads move to problem p's record
  __device__ void set_record(int64_t p) {
    gdbl* r = rec0 + p * L.r_total;
    Hm = r + L.r_h;
    Ap = r + L.r_ap;
    At = r + L.r_at;
    Tm = r + L.r_t;
    Sm = r + L.r_s;
    Vr = r + L.r_v;
  }

  // setup_iter's cone state for the later solve_kkt calls (densesolver.jl:41-52
  // keeps it in the solver object): LAM WB CA, the per-cone constants, sing.
  // The matrices (Li, A, Li A', S^-1) stay where factor() left them: with a
  // record buffer (set_record) they are the problem's own; X, the pivot rows
  // and 1/d stay in the workgroup's scratch slot.
  __device__ void store_record() {
    const int KP = L.KP;
    for (int i = tid; i < KP; i += NTH) {
      Vr[i] = LV(LAM + i);
      Vr[KP + i] = LV(WB + i);
      Vr[2 * KP + i] = LV(CA + i);
    }
    for (int i = tid; i < 12 * MAXC; i += NTH) Vr[3 * KP + i] = LV(L.o_cc + i);
    if (tid == 0) Vr[3 * KP + 12 * MAXC] = sing ? 1.0 : 0.0;
    BAR();
  }
  __device__ void load_record() {
    const int KP = L.KP;
    for (int i = tid; i < KP; i += NTH) {
      LV(LAM + i) = Vr[i];
      LV(WB + i) = Vr[KP + i];
      LV(CA + i) = Vr[2 * KP + i];
    }
    for (int i = tid; i < 12 * MAXC; i += NTH) LV(L.o_cc + i) = Vr[3 * KP + i];
    sing = __builtin_amdgcn_readfirstlane((int)Vr[3 * KP + 12 * MAXC]) != 0;
    BAR();
  }

  __device__ __forceinline__ double ccv(int q, int c) const { return LV(L.o_cc + q * MAXC + c); }
  __device__ __forceinline__ void ccset(int q, int c, double v) { LV(L.o_cc + q * MAXC + c) = v; }
  __device__ __forceinline__ double e_of(int i) const {
    const int t = (int)LV(L.o_rc + i) & 3;
    return (t == 0 || t == 1) ? 1.0 : 0.0;
  }

  __device__ double block_sum(double v) {
    v = wave_sum(v);
    BAR();
    if (lane == 0) LV(L.o_red + wv) = v;
    BAR();
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < NW; ++w) t += LV(L.o_red + w);
    return t;
  }
  __device__ double block_max(double v) {
    v = wave_max(v);
    BAR();
    if (lane == 0) LV(L.o_red + wv) = v;
    BAR();
    double t = -INFINITY;
#pragma unroll
    for (int w = 0; w < NW; ++w) t = fmax(t, LV(L.o_red + w));
    return t;
  }
  __device__ bool block_any(bool v) { return block_max(v ? 1.0 : 0.0) > 0.0; }

  // ---------------------------------------------------------------- setup
  __device__ void init_tables() {
    for (int i = tid; i < L.KP; i += NTH) {
      int code = 3;
      if (i < k)
        for (int c = 0; c < nc; ++c) {
          const int o = a.cones.offs[c], d = a.cones.dim[c];
          if (i >= o && i < o + d) {
            code = c * 4 + (a.cones.kind[c] == POC_K ? 0 : (i == o ? 1 : 2));
            break;
          }
        }
      LV(L.o_rc + i) = (double)code;
    }
    if (tid < 32) LV(L.o_red + 16 + tid) = 0.0;  // all-zero bits: the u64 stamp totals start at 0
    BAR();
    st_last = __builtin_amdgcn_s_memtime();
  }
  __device__ void flush_stamps() {
#ifdef SOCP_DIAG
    BAR();
    if (!GV && tid == 0 && a.stamps) {
      const unsigned long long* st = reinterpret_cast<const unsigned long long*>(lg_lds + L.o_red + 16);
      for (int i = 0; i <= NSTAMP + NSUBSTAMP; ++i) atomicAdd(a.stamps + i, st[i]);
    }
#endif
  }

  __device__ void load(int64_t p) {
    Gp = (gcdbl*)a.G + p * (int64_t)k * n;
    for (int e = tid; e < 7 * L.KP; e += NTH) LV(L.o_kvd + e) = 0.0;
    for (int e = tid; e < 8 * L.KP; e += NTH) LV(L.o_kvl + e) = 0.0;
    for (int e = tid; e < 6 * L.NPAD + 5 * L.MPAD; e += NTH) LV(L.o_nv + e) = 0.0;
    BAR();
    for (int j = tid; j < n; j += NTH) LV(C_ + j) = a.c[p * n + j];
    for (int i = tid; i < m; i += NTH) LV(B_ + i) = a.b[p * m + i];
    for (int i = tid; i < k; i += NTH) LV(H_ + i) = a.h[p * k + i];
    const double* Ag = a.A + p * (int64_t)m * n;
    const int NP = L.NPAD, MP = L.MPAD;
    for (int e = tid; e < MP * NP; e += NTH) {
      const int j = e / MP, r = e - j * MP;
      double v = 0.0;
      if (r < m && j < n) v = Ag[(int64_t)j * m + r];
      Ap[e] = v;
    }
    for (int e = tid; e < MP * NP; e += NTH) {
      const int r = e / NP, j = e - r * NP;
      double v = 0.0;
      if (r < m && j < n) v = Ag[(int64_t)j * m + r];
      At[e] = v;
    }
    BAR();
  }

  // W = I: the initial-point system (solver.jl:68-84) is the KKT system with
  // W = I, lambda = e, ds = 0.
  __device__ void scaling_identity() {
    for (int i = tid; i < k; i += NTH) {
      const double e = e_of(i);
      LV(WB + i) = e;
      LV(LAM + i) = e;
      LV(CA + i) = 1.0;
    }
    for (int c = tid; c < nc; c += NTH) {
      ccset(CC_MU, c, 1.0);
      ccset(CC_IMU, c, 1.0);
      ccset(CC_WB0, c, 1.0);
      ccset(CC_I1, c, 0.5);
      ccset(CC_W2, c, 0.0);
      ccset(CC_L0, c, 1.0);
      ccset(CC_AA, c, 1.0);
      ccset(CC_IAA, c, 1.0);
      ccset(CC_IL0, c, 1.0);
      ccset(CC_IL0AA, c, 1.0);
      ccset(CC_SA, c, 1.0);
      ccset(CC_SAL, c, 0.5);
    }
    BAR();
  }

  // ------------------------------------------------------ cone vector ops
  // POC elements are elementwise over all threads; SOC cone c belongs to
  // wavefront (c - csoc) % 8, whose lanes stride over the cone's elements and
  // reduce its dot products with wave_sum.  Formulas: the register kernel's.

  // compute_scaling (scalings.jl:22-110) and ds = lam o lam (solver.jl:120)
  __device__ bool scaling_op(double& ll, bool& dm_aa, bool write_ds) {
    double llp = 0.0;
    bool dm = false, da = false;
    for (int i = tid; i < kpoc; i += NTH) {
      const double s = LV(S_ + i), z = LV(Z_ + i);
      const double r = s / z, pr = s * z, ir = z / s;
      dm |= (r < 0.0) || (pr < 0.0) || (ir < 0.0);
      const double li = sqrt(pr);
      LV(WB + i) = sqrt(r);
      LV(LAM + i) = li;
      LV(CA + i) = sqrt(ir);
      if (write_ds) LV(DS + i) = li * li;
      llp += li * li;
    }
    for (int c = csoc + wv; c < nc; c += NW) {
      const int o = a.cones.offs[c], d = a.cones.dim[c];
      const double z0 = LV(Z_ + o), s0 = LV(S_ + o);
      double pz = 0.0, ps = 0.0, pzs = 0.0;
      for (int i = o + 1 + lane; i < o + d; i += 64) {
        const double zi = LV(Z_ + i), si = LV(S_ + i);
        pz += zi * zi;
        ps += si * si;
        pzs += zi * si;
      }
      const double vz = wave_sum(pz), vs = wave_sum(ps), vzs = wave_sum(pzs);
      const double onrmz = z0 * z0 - vz, onrms = s0 * s0 - vs;
      const double nrmz = sqrt(onrmz), nrms = sqrt(onrms);
      const double fz = 1.0 / nrmz, fs = 1.0 / nrms;
      const double zb0 = z0 * fz, sb0 = s0 * fs;
      const double nsum = zb0 * sb0 + vzs * fz * fs;
      const double garg = (1.0 + nsum) / 2.0;
      const double gamma = sqrt(garg);
      const double fg = 1.0 / (2.0 * gamma);
      const double wb0 = (sb0 + zb0) * fg;
      const double ratio = nrms / nrmz, prod = nrms * nrmz;
      const double mu = sqrt(ratio), tmv1 = sqrt(prod);
      const double mult = tmv1 / (zb0 + sb0 + 2.0 * gamma);
      const double l0 = gamma * tmv1;
      const double im = 1.0 / mu;
      dm |= (onrmz < 0.0) || (onrms < 0.0) || (garg < 0.0) || (ratio < 0.0) || (prod < 0.0);
      double pl = 0.0, pw = 0.0;
      for (int i = o + 1 + lane; i < o + d; i += 64) {
        const double zbi = LV(Z_ + i) * fz, sbi = LV(S_ + i) * fs;
        const double w = (sbi - zbi) * fg;
        const double li = (sbi * (gamma + zb0) + zbi * (gamma + sb0)) * mult;
        LV(WB + i) = w;
        LV(LAM + i) = li;
        if (write_ds) LV(DS + i) = l0 * li + l0 * li;
        pl += li * li;
        pw += w * w;
      }
      const double v1 = wave_sum(pl), v2 = wave_sum(pw);
      const double v0 = l0 * l0 + v1;  // lam'lam of the cone (vprod!'s head, vectors.jl:66)
      const double aa = l0 * l0 - v1;  // iprod!'s a (vectors.jl:105)
      da |= aa < 0.0;
      if (lane == 0) {
        LV(WB + o) = wb0;
        LV(LAM + o) = l0;
        if (write_ds) LV(DS + o) = v0;
        const double sa = 1.0 / sqrt(aa);
        ccset(CC_MU, c, mu);
        ccset(CC_IMU, c, im);
        ccset(CC_WB0, c, wb0);
        ccset(CC_I1, c, 1.0 / (1.0 + wb0));
        ccset(CC_W2, c, v2);
        ccset(CC_L0, c, l0);
        ccset(CC_AA, c, aa);
        ccset(CC_IAA, c, 1.0 / aa);
        ccset(CC_IL0, c, 1.0 / l0);
        ccset(CC_IL0AA, c, 1.0 / (l0 * aa));
        ccset(CC_SA, c, sa);
        ccset(CC_SAL, c, 1.0 / (sa * l0 + 1.0));
        llp += v0;
      }
    }
    ll = block_sum(llp);
    dm_aa = block_any(da);
    return block_any(dm);
  }

  // First half of solve_kkt (densesolver.jl:61-66): k0 = lam^-1 o ds, k1 = W k0,
  // k2 = dz - k1, T2 = W^-1 W^-1 k2.  In: DS, DZ.  Out: K0, K2, T2.
  __device__ void solve_head() {
    for (int i = tid; i < kpoc; i += NTH) {
      const double k0 = LV(DS + i) / LV(LAM + i);
      const double k2 = LV(DZ + i) - LV(WB + i) * k0;
      const double ca = LV(CA + i);
      LV(K0 + i) = k0;
      LV(K2 + i) = k2;
      LV(T2 + i) = ca * (ca * k2);
    }
    for (int c = csoc + wv; c < nc; c += NW) {
      const int o = a.cones.offs[c], d = a.cones.dim[c];
      const double x0 = LV(DS + o);
      double pt = 0.0;
      for (int i = o + 1 + lane; i < o + d; i += 64) pt = fma(LV(LAM + i), LV(DS + i), pt);
      const double t = wave_sum(pt);
      const double l0 = ccv(CC_L0, c), iaa = ccv(CC_IAA, c), il0 = ccv(CC_IL0, c), il0aa = ccv(CC_IL0AA, c);
      const double k00 = (x0 * l0 - t) * iaa;
      double pd = 0.0;
      for (int i = o + 1 + lane; i < o + d; i += 64) {
        const double lam = LV(LAM + i);
        const double k0 = -(x0 * lam * iaa) + LV(DS + i) * il0 + lam * t * il0aa;
        LV(K0 + i) = k0;
        pd = fma(LV(WB + i), k0, pd);
      }
      const double del = wave_sum(pd);
      const double mu = ccv(CC_MU, c), wb0 = ccv(CC_WB0, c), i1 = ccv(CC_I1, c);
      const double k10 = mu * (wb0 * k00 + del);
      const double k20 = LV(DZ + o) - k10;
      double pa = 0.0;
      for (int i = o + 1 + lane; i < o + d; i += 64) {
        const double wb = LV(WB + i);
        const double k2 = LV(DZ + i) - mu * (LV(K0 + i) + (k00 + del * i1) * wb);
        LV(K2 + i) = k2;
        pa = fma(wb, k2, pa);
      }
      const double a1 = wave_sum(pa);
      const double im = ccv(CC_IMU, c), w2 = ccv(CC_W2, c);
      const double cy = a1 * i1 - k20;
      const double y0 = im * (wb0 * k20 - a1);
      const double a2 = im * (a1 + cy * w2);
      for (int i = o + 1 + lane; i < o + d; i += 64) {
        const double wb = LV(WB + i);
        const double y = im * (LV(K2 + i) + cy * wb);
        LV(T2 + i) = im * (y + (a2 * i1 - y0) * wb);
      }
      if (lane == 0) {
        LV(K0 + o) = k00;
        LV(K2 + o) = k20;
        LV(T2 + o) = im * (wb0 * y0 - a2);
      }
    }
    BAR();
  }

  // Second half of solve_kkt (densesolver.jl:83-88) and, with do_step,
  // compute_step (mats.jl:30-86) of the direction: kt3 = W rz (T1) and
  // kt2 = W^-1 rs (K0) come out of the solve.  In: K1, K0.  Out: RZ, RS, T1, K0.
  __device__ double solve_tail(bool do_step, bool dm_aa, int& dom) {
    double mx = -INFINITY;
    for (int i = tid; i < kpoc; i += NTH) {
      const double ca = LV(CA + i), y = ca * LV(K1 + i);
      const double kn = LV(K0 + i) - y;
      LV(RZ + i) = ca * y;
      LV(RS + i) = LV(WB + i) * kn;
      LV(T1 + i) = y;
      LV(K0 + i) = kn;
      const double lam = LV(LAM + i);
      mx = fmax(mx, fmax(-y / lam, -kn / lam));
    }
    for (int c = csoc + wv; c < nc; c += NW) {
      const int o = a.cones.offs[c], d = a.cones.dim[c];
      const double k10 = LV(K1 + o);
      double p1 = 0.0;
      for (int i = o + 1 + lane; i < o + d; i += 64) p1 = fma(LV(WB + i), LV(K1 + i), p1);
      const double a1 = wave_sum(p1);
      const double im = ccv(CC_IMU, c), wb0 = ccv(CC_WB0, c), i1 = ccv(CC_I1, c), w2 = ccv(CC_W2, c);
      const double mu = ccv(CC_MU, c);
      const double cy = a1 * i1 - k10;
      const double y0 = im * (wb0 * k10 - a1);
      const double a2 = im * (a1 + cy * w2);
      const double kn0 = LV(K0 + o) - y0;
      double pd = 0.0;
      for (int i = o + 1 + lane; i < o + d; i += 64) {
        const double wb = LV(WB + i);
        const double y = im * (LV(K1 + i) + cy * wb);
        const double kn = LV(K0 + i) - y;
        LV(RZ + i) = im * (y + (a2 * i1 - y0) * wb);
        LV(T1 + i) = y;
        LV(K0 + i) = kn;
        pd = fma(wb, kn, pd);
      }
      const double del = wave_sum(pd);
      for (int i = o + 1 + lane; i < o + d; i += 64)
        LV(RS + i) = mu * (LV(K0 + i) + (kn0 + del * i1) * LV(WB + i));
      if (lane == 0) {
        LV(RZ + o) = im * (wb0 * y0 - a2);
        LV(RS + o) = mu * (wb0 * kn0 + del);
        LV(T1 + o) = y0;
        LV(K0 + o) = kn0;
      }
      if (do_step) {  // scmax (mats.jl:42-86) of kt3 and kt2
        double pw0 = 0.0, pw1 = 0.0;
        for (int i = o + 1 + lane; i < o + d; i += 64) {
          const double lam = LV(LAM + i);
          pw0 = fma(lam, LV(T1 + i), pw0);
          pw1 = fma(lam, LV(K0 + i), pw1);
        }
        const double w0 = wave_sum(pw0), w1 = wave_sum(pw1);
        const double sa = ccv(CC_SA, c), l0 = ccv(CC_L0, c), sal = ccv(CC_SAL, c);
        const double r1y = sa * l0 * y0 - sa * w0, r1k = sa * l0 * kn0 - sa * w1;
        const double cyy = (r1y + y0) * sal, cyk = (r1k + kn0) * sal;
        double qy = 0.0, qk = 0.0;
        for (int i = o + 1 + lane; i < o + d; i += 64) {
          const double lam = LV(LAM + i);
          const double ty = sa * (LV(T1 + i) - cyy * sa * lam), tk = sa * (LV(K0 + i) - cyk * sa * lam);
          qy = fma(ty, ty, qy);
          qk = fma(tk, tk, qk);
        }
        const double vy = sqrt(wave_sum(qy)) - sa * r1y, vk = sqrt(wave_sum(qk)) - sa * r1k;
        mx = fmax(mx, fmax(vy, vk));
      }
    }
    if (!do_step) {
      BAR();
      return 0.0;
    }
    const double t = fmax(block_max(mx), 0.0);
    dom = dm_aa ? 1 : 0;
    return (t == 0.0) ? 1.0 : fmin(1.0, 1.0 / t);
  }

  // rho, sigma, mu (solver.jl:132-134) and the corrector right-hand side
  // (:136-140).  In: K0 (kt2), T1 (kt3), DS, DZ, RD, RP.
  __device__ void affine_post(double tstep, double ll) {
    double pk = 0.0;
    for (int i = tid; i < k; i += NTH) pk = fma(LV(K0 + i), LV(T1 + i), pk);
    const double kk = block_sum(pk);
    const double t = tstep;
    const double rho = 1.0 - t - t * t * kk / ll;
    const double cr = isnan(rho) ? rho : (rho < 0.0 ? 0.0 : (rho > 1.0 ? 1.0 : rho));
    const double sig = ipow(cr, a.sigma_exp);  // max(0,min(1,rho))^3 (solver.jl:133)
    const double mu_ipm = ll / a.deg;
    const double scf = 1.0 - sig;
    for (int i = tid; i < kpoc; i += NTH) LV(DS + i) = LV(DS + i) + (sig * mu_ipm - LV(K0 + i) * LV(T1 + i));
    for (int c = csoc + wv; c < nc; c += NW) {
      const int o = a.cones.offs[c], d = a.cones.dim[c];
      double ph = 0.0;
      for (int i = o + lane; i < o + d; i += 64) ph = fma(LV(K0 + i), LV(T1 + i), ph);
      const double hsum = wave_sum(ph);
      const double a20 = LV(K0 + o), a30 = LV(T1 + o);
      for (int i = o + 1 + lane; i < o + d; i += 64)
        LV(DS + i) = LV(DS + i) - (a20 * LV(T1 + i) + a30 * LV(K0 + i));
      if (lane == 0) LV(DS + o) = LV(DS + o) + (sig * mu_ipm - hsum);
    }
    for (int i = tid; i < k; i += NTH) LV(DZ + i) = LV(DZ + i) * scf;
    for (int j = tid; j < n; j += NTH) LV(RD + j) = LV(RD + j) * scf;
    for (int i = tid; i < m; i += NTH) LV(RP + i) = LV(RP + i) * scf;
    BAR();
  }

  // max_step(-iz), max_step(iz) (mats.jl:1-28) for the initial shift (solver.jl:88-101)
  __device__ void maxstep_op(int xv, double& alphp, double& alphd) {
    double mp = -INFINITY, md = -INFINITY;
    for (int i = tid; i < kpoc; i += NTH) {
      const double x = LV(xv + i);
      mp = fmax(mp, x);
      md = fmax(md, -x);
    }
    for (int c = csoc + wv; c < nc; c += NW) {
      const int o = a.cones.offs[c], d = a.cones.dim[c];
      double pq = 0.0;
      for (int i = o + 1 + lane; i < o + d; i += 64) pq = fma(LV(xv + i), LV(xv + i), pq);
      const double nr = sqrt(wave_sum(pq)), x0 = LV(xv + o);
      mp = fmax(mp, nr + x0);
      md = fmax(md, nr - x0);
    }
    alphp = block_max(mp);
    alphd = block_max(md);
  }

  // ---------------------------------------------------------- dense blocks
  // acc[ta][tb] += sum_kk P[kk][I0+16ta+i] * Q[kk][J0+16tb+j] over kk < kr, where
  // P[kk][col] sits at P[col*ld + kk] (column-major, k index fastest).  At MFMA
  // step s, lane group g feeds k-row k0 + 4g + s (the k order is free), so a
  // lane's operands are 4 consecutive doubles (two 16-byte loads).  qs >= 0:
  // the Q operand of k-row kk is scaled by LDS[qs + kk].
  // LO: a diagonal block, whose tiles above the diagonal are not needed (skipped)
  template <bool LO = false>
  __device__ __forceinline__ void blk_gemm(d4 (&acc)[4][4], gcdbl* P, gcdbl* Q, int ld, int I0,
                                           int J0, int kr, bool same, int qs) {
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll SOCP_LG_SYRK_UNROLL
    for (int k0 = 0; k0 < kr; k0 += 16) {
      double av[4][4], bv[4][4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        gcdbl2* pa = reinterpret_cast<gcdbl2*>(P + (int64_t)(I0 + 16 * t + cl) * ld + k0 + 4 * g);
        const dbl2 x0 = pa[0], x1 = pa[1];
        av[t][0] = x0.x;
        av[t][1] = x0.y;
        av[t][2] = x1.x;
        av[t][3] = x1.y;
      }
      if (same) {
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int s = 0; s < 4; ++s) bv[t][s] = av[t][s];
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          gcdbl2* pb = reinterpret_cast<gcdbl2*>(Q + (int64_t)(J0 + 16 * t + cl) * ld + k0 + 4 * g);
          const dbl2 x0 = pb[0], x1 = pb[1];
          bv[t][0] = x0.x;
          bv[t][1] = x0.y;
          bv[t][2] = x1.x;
          bv[t][3] = x1.y;
        }
      }
      if (qs >= 0) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          const double f = LV(qs + k0 + 4 * g + s);
#pragma unroll
          for (int t = 0; t < 4; ++t) bv[t][s] *= f;
        }
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int ta = 0; ta < 4; ++ta)
#pragma unroll
          for (int tb = 0; tb < 4; ++tb)
            if (!LO || tb <= ta) acc[ta][tb] = mfma(av[ta][s], bv[tb][s], acc[ta][tb]);
    }
  }

  // The sweep's deferred Gram update, acc += sum_{c<64} Y[c][I-slice]' (fv[c]
  // Y[c][J-slice]) for the row-major 64-row panel Y (row c at Y + c*ld), in the
  // transposed MFMA orientation: acc[a][b] (lane (g, cl),
  // register r) holds block element (I0 + 16b + cl, J0 + 16a + g + 4r), so the
  // column-major read-modify-write of the block is 128 contiguous bytes per
  // 16 lanes (load_blkT / store_blkT) instead of 32 bytes over 16 columns.
  // LO (diagonal block): tiles with b < a lie above the diagonal (skipped).
  template <bool LO = false, bool FV = true>
  __device__ __forceinline__ void gram_blkT(d4 (&acc)[4][4], gcdbl* Y, int ld, int I0, int J0, gcdbl* fv) {
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll SOCP_LG_GRAM_UNROLL
    for (int k0 = 0; k0 < 64; k0 += 16) {
      double av[4][4], bv[4][4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        gcdbl* row = Y + (int64_t)(k0 + 4 * s + g) * ld;
        const double f = FV ? fv[k0 + 4 * s + g] : 1.0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          av[t][s] = f * row[J0 + 16 * t + cl];
          bv[t][s] = row[I0 + 16 * t + cl];
        }
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int a_ = 0; a_ < 4; ++a_)
#pragma unroll
          for (int b_ = 0; b_ < 4; ++b_)
            if (!LO || b_ >= a_) acc[a_][b_] = mfma(av[a_][s], bv[b_][s], acc[a_][b_]);
    }
  }
  // one 16-column group a_ of the block (acc[a_][*] of gram_blkT): the same
  // MFMAs in the same order, so a block split into its four column groups over
  // four wavefronts gives gram_blkT's result bit for bit
  template <bool LO = false>
  __device__ __forceinline__ void gram_colT(d4 (&acc)[4], gcdbl* Y, int ld, int I0, int J0, gcdbl* fv, int a_) {
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll 2
    for (int k0 = 0; k0 < 64; k0 += 16) {
      double av[4], bv[4][4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        gcdbl* row = Y + (int64_t)(k0 + 4 * s + g) * ld;
        av[s] = fv[k0 + 4 * s + g] * row[J0 + 16 * a_ + cl];
#pragma unroll
        for (int t = 0; t < 4; ++t) bv[t][s] = row[I0 + 16 * t + cl];
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int b_ = 0; b_ < 4; ++b_)
          if (!LO || b_ >= a_) acc[b_] = mfma(av[s], bv[b_][s], acc[b_]);
    }
  }
  template <bool LO = false>
  __device__ __forceinline__ void load_colT(d4 (&acc)[4], gcdbl* M, int ld, int I0, int J0, int a_) {
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int b_ = 0; b_ < 4; ++b_)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        acc[b_][r] = (LO && b_ < a_) ? 0.0 : M[(int64_t)(J0 + 16 * a_ + g + 4 * r) * ld + I0 + 16 * b_ + cl];
  }
  template <bool LO = false>
  __device__ __forceinline__ void store_colT(const d4 (&acc)[4], gdbl* M, int ld, int I0, int J0, int a_) {
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int b_ = 0; b_ < 4; ++b_)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (!LO || b_ >= a_) M[(int64_t)(J0 + 16 * a_ + g + 4 * r) * ld + I0 + 16 * b_ + cl] = acc[b_][r];
  }
  template <bool LO = false>
  __device__ __forceinline__ void load_blkT(d4 (&acc)[4][4], gcdbl* M, int ld, int I0, int J0) {
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int a_ = 0; a_ < 4; ++a_)
#pragma unroll
      for (int b_ = 0; b_ < 4; ++b_)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          acc[a_][b_][r] = (LO && b_ < a_) ? 0.0 : M[(int64_t)(J0 + 16 * a_ + g + 4 * r) * ld + I0 + 16 * b_ + cl];
  }
  template <bool LO = false>
  __device__ __forceinline__ void store_blkT(const d4 (&acc)[4][4], gdbl* M, int ld, int I0, int J0) {
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int a_ = 0; a_ < 4; ++a_)
#pragma unroll
      for (int b_ = 0; b_ < 4; ++b_)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (LO && b_ < a_) continue;
          M[(int64_t)(J0 + 16 * a_ + g + 4 * r) * ld + I0 + 16 * b_ + cl] = acc[a_][b_][r];
        }
  }

  // 64x64 block (I0, J0) of a column-major matrix <-> the f64 MFMA C/D layout
  // (lane (g, cl) holds rows g + 4r, column cl of each 16x16 tile)
  template <bool LO = false>
  __device__ __forceinline__ void load_blk(d4 (&acc)[4][4], gcdbl* M, int ld, int I0, int J0) {
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int ta = 0; ta < 4; ++ta)
#pragma unroll
      for (int tb = 0; tb < 4; ++tb)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          acc[ta][tb][r] = (LO && tb > ta) ? 0.0 : M[(int64_t)(J0 + 16 * tb + cl) * ld + I0 + 16 * ta + g + 4 * r];
  }
  // idpad: diagonal entries at index >= idpad are set to 1 (identity padding)
  template <bool LO = false>
  __device__ __forceinline__ void store_blk(const d4 (&acc)[4][4], gdbl* M, int ld, int I0, int J0, int idpad) {
    const int g = lane >> 4, cl = lane & 15;
#pragma unroll
    for (int ta = 0; ta < 4; ++ta)
#pragma unroll
      for (int tb = 0; tb < 4; ++tb)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (LO && tb > ta) continue;
          const int R = I0 + 16 * ta + g + 4 * r, Cc = J0 + 16 * tb + cl;
          const double v = (R == Cc && R >= idpad) ? 1.0 : acc[ta][tb][r];
          M[(int64_t)Cc * ld + R] = v;
        }
  }
  __device__ __forceinline__ static void zero_blk(d4 (&acc)[4][4]) {
#pragma unroll
    for (int ta = 0; ta < 4; ++ta)
#pragma unroll
      for (int tb = 0; tb < 4; ++tb) acc[ta][tb] = (d4){0.0, 0.0, 0.0, 0.0};
  }
  // lower-triangle block index t -> (I, J), I >= J
  __device__ __forceinline__ static void tri_ij(int t, int& I, int& J) {
    I = 0;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    J = t - I * (I + 1) / 2;
  }

  // X[:, j] = W^-1 G[:, j] (iscale!, scalings.jl:145-173) for every column:
  // a wavefront takes CG columns at a time (independent per-cone reductions
  // overlap).  Zero padding (rows >= k, columns >= n).
  // W^-1 G fast path (at most FX_NC SOC cones, k <= 64 * FX_R; any POC block):
  // a wavefront takes FX_CG columns at a time and loads them whole (one HBM
  // round trip per pass), reduces every cone's wbar-weighted tail sum from
  // registers, and writes the columns of X.  Otherwise form_X.
#ifndef SOCP_LG_FX_CG
#define SOCP_LG_FX_CG 4  // W^-1 G fast path: columns per wavefront pass (2: +2.4 ms at C4, round 5)
#endif
  static constexpr int FX_CG = SOCP_LG_FX_CG, FX_NC = 8, FX_R = 10;
  static_assert(FX_CG * FX_NC <= 32, "per-wavefront fx slots: 32 sums, then 32 head values");
  __device__ bool form_X_fast_ok() const { return nc - csoc <= FX_NC && (k + 63) / 64 <= FX_R; }
  // chunked: X in 4-row chunks, chunk-major -- X[i][j] at ((i/4) NPAD + j) 4 + i%4
  // -- so a chunk is one contiguous 32 NPAD-byte run (the staged SYRK's DMA)
  // 32 values per lane -> value q summed over the wavefront, in lanes 2q, 2q+1
  // (v[0] on return)
  __device__ __forceinline__ void fx_reduce_scatter(double (&v)[32]) const {
    auto swap_add = [](double& x, double& y, bool rows) {
      // x' = [x.lo, y.lo], y' = [x.hi, y.hi] (halves of the wave or of each 32-lane half)
      const unsigned xl = (unsigned)__double2loint(x), xh = (unsigned)__double2hiint(x);
      const unsigned yl = (unsigned)__double2loint(y), yh = (unsigned)__double2hiint(y);
      const auto l = rows ? __builtin_amdgcn_permlane16_swap(xl, yl, false, false)
                          : __builtin_amdgcn_permlane32_swap(xl, yl, false, false);
      const auto h = rows ? __builtin_amdgcn_permlane16_swap(xh, yh, false, false)
                          : __builtin_amdgcn_permlane32_swap(xh, yh, false, false);
      x = __hiloint2double((int)h[0], (int)l[0]) + __hiloint2double((int)h[1], (int)l[1]);
    };
#pragma unroll
    for (int j = 0; j < 16; ++j) swap_add(v[j], v[j + 16], false);  // lanes >= 32 now carry j + 16
#pragma unroll
    for (int j = 0; j < 8; ++j) swap_add(v[j], v[j + 8], true);  // odd rows carry j + 8
    const int ln = lane;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bool up = ln & 8;
      const double send = up ? v[j] : v[j + 4], keep = up ? v[j + 4] : v[j];
      v[j] = keep + row_partner<8>(send);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const bool up = ln & 4;
      const double send = up ? v[j] : v[j + 2], keep = up ? v[j + 2] : v[j];
      v[j] = keep + row_partner<4>(send);
    }
    {
      const bool up = ln & 2;
      const double send = up ? v[0] : v[1], keep = up ? v[1] : v[0];
      v[0] = keep + row_partner<2>(send);
    }
    v[0] += row_partner<1>(v[0]);
  }
  __device__ bool form_X_fast(bool chunked) {
    const int nsoc = nc - csoc;
    const int R = (k + 63) / 64;
    if (!form_X_fast_ok()) return false;
    const int NPD = L.NPAD;
    const int KP = L.KP, ln = lane, kk = k, nn = n;
    const int fx = L.o_fx + wv * 64;  // [0,32): del[u][c], [32,64): head value g0[u][c]
    double wbr[FX_R];
#pragma unroll
    for (int r = 0; r < FX_R; ++r) {
      const int row = ln + 64 * r;
      wbr[r] = (r < R && row < kk) ? LV(WB + row) : 0.0;
    }
    // columns j0 .. j0 + FX_CG - 1 of G into gv (dead columns read column 0)
    auto load_cols = [&](double (&dst)[FX_CG][FX_R], int j0_) {
      const int nl_ = nn - j0_;
      gcdbl* gp = Gp + (int64_t)(j0_ < nn ? j0_ : 0) * kk;
#pragma unroll
      for (int r = 0; r < FX_R; ++r) {
        const int row = ln + 64 * r;
        const bool in = r < R && row < kk;
#pragma unroll
        for (int u = 0; u < FX_CG; ++u) dst[u][r] = in ? gp[(int64_t)(u < nl_ ? u : 0) * kk + row] : 0.0;
      }
    };
    // (the next group's loads issued before this group's reductions, from a
    // second buffer, measured 1 % slower at C4)
    double gv[FX_CG][FX_R];
    for (int j0 = FX_CG * wv; j0 < L.NPAD; j0 += FX_CG * NW) {
      const int nl = nn - j0;
      gcdbl* g0p = Gp + (int64_t)(j0 < nn ? j0 : 0) * kk;
      gdbl* x0 = Xw + (int64_t)j0 * KP;
      load_cols(gv, j0);
#if SOCP_LG_FX_RS
      double rsv[FX_CG * FX_NC];  // slot u * FX_NC + ci: this lane's partial of del
#pragma unroll
      for (int q = 0; q < FX_CG * FX_NC; ++q) rsv[q] = 0.0;
#endif
      // per SOC cone: del = sum over the tail of wbar_i G_ij
#pragma unroll
      for (int ci = 0; ci < FX_NC; ++ci) {
        if (ci >= nsoc) break;
        const int c = csoc + ci, o = a.cones.offs[c], d = a.cones.dim[c];
        double pd[FX_CG];
#pragma unroll
        for (int u = 0; u < FX_CG; ++u) pd[u] = 0.0;
#pragma unroll
        for (int r = 0; r < FX_R; ++r) {
          const int row = ln + 64 * r;
          const double w = (row > o && row < o + d) ? wbr[r] : 0.0;
#pragma unroll
          for (int u = 0; u < FX_CG; ++u) pd[u] = fma(w, gv[u][r], pd[u]);
        }
#if SOCP_LG_FX_RS
#pragma unroll
        for (int u = 0; u < FX_CG; ++u) rsv[u * FX_NC + ci] = pd[u];
#endif
        // the head value G[o][j0 + u] is already in a register (row o of the
        // loaded columns: lane o % 64, slot o / 64): a readlane instead of a
        // global load per column and cone on the wave's critical path
        const int ro = o >> 6, lo = o & 63;
#pragma unroll
        for (int u = 0; u < FX_CG; ++u) {
          double gh = 0.0;
          if constexpr (!XI) {  // (the explicit-inverse kernel spills with it: a global load there)
#pragma unroll
            for (int r = 0; r < FX_R; ++r)
              if (r == ro) gh = readlane_d(gv[u][r], lo);  // wave-uniform branch
          } else {
            gh = g0p[(int64_t)(u < nl ? u : 0) * kk + o];
          }
#if SOCP_LG_FX_RS
          if (ln == 0) LV(fx + 32 + u * FX_NC + ci) = gh;
#else
#if SOCP_LG_KO & 1  // timing knock-out (tuning builds only; results wrong): no reductions
          const double del = pd[u];
#else
          const double del = wave_sum(pd[u]);
#endif
          if (ln == 0) {
            LV(fx + u * FX_NC + ci) = del;
            LV(fx + 32 + u * FX_NC + ci) = gh;
          }
#endif
        }
      }
#if SOCP_LG_FX_RS
      // the 32 sums at once by a reduce-scatter over the wavefront: each level
      // halves the values a lane carries and doubles the lanes each covers
      // (lanes +-32 and +-16 by permlane swaps, +-8, +-4, +-2 by DPP, +-1 an
      // all-reduce step), so that sum q ends in lanes 2q and 2q + 1 -- 124
      // instructions instead of 32 wave-wide all-reduces
      fx_reduce_scatter(rsv);
      if ((ln & 1) == 0) LV(fx + (ln >> 1)) = rsv[0];
#endif
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int r = 0; r < FX_R; ++r) {
        const int row = ln + 64 * r;
        if (r * 64 >= KP) break;
        const int code = row < kk ? (int)LV(L.o_rc + row) : 3;
        const int c = code >> 2, typ = code & 3, ci = c - csoc;
        const bool soc = typ == 1 || typ == 2;
        const double ca = typ == 0 ? LV(CA + row) : 0.0;
        const double im = soc ? ccv(CC_IMU, c) : 0.0, wb0 = soc ? ccv(CC_WB0, c) : 0.0,
                     i1 = soc ? ccv(CC_I1, c) : 0.0;
#pragma unroll
        for (int u = 0; u < FX_CG; ++u) {
          const double del = soc ? LV(fx + u * FX_NC + ci) : 0.0, gh = soc ? LV(fx + 32 + u * FX_NC + ci) : 0.0;
          const double g = gv[u][r];
          double x = 0.0;
          if (typ == 0) x = ca * g;
          if (typ == 1) x = im * (wb0 * g - del);
          if (typ == 2) x = im * (g + (-gh + del * i1) * wbr[r]);
          if (u >= nl) x = 0.0;
          if (row < KP && !((SOCP_LG_KO & 2) && x != 1.2345)) {  // KO 2: no X stores (tuning builds only)
            if (chunked)
              Xw[((int64_t)(row >> 2) * NPD + j0 + u) * 4 + (row & 3)] = x;
            else
              x0[u * KP + row] = x;
          }
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    BAR();
    return true;
  }

  __device__ void form_X() {
    const int KP = L.KP, ln = lane, kk = k, nn = n;
    for (int j0 = CG * wv; j0 < L.NPAD; j0 += CG * NW) {
      // column j0 + u of G at g0 + u*k, of X at x0 + u*KP (dead columns read column 0)
      gcdbl* g0 = Gp + (int64_t)(j0 < nn ? j0 : 0) * kk;
      gdbl* x0 = Xw + (int64_t)j0 * KP;
      const int nl = nn - j0;  // live columns: u < nl
#define GC(u, i) g0[(int64_t)((u) < nl ? (u) : 0) * kk + (i)]
      for (int i = ln; i < kpoc; i += 64) {
        const double ca = LV(CA + i);
#pragma unroll
        for (int u = 0; u < CG; ++u) x0[u * KP + i] = (u < nl) ? ca * GC(u, i) : 0.0;
      }
      for (int c = csoc; c < nc; ++c) {
        const int o = a.cones.offs[c], d = a.cones.dim[c];
        double pd[CG];
#pragma unroll
        for (int u = 0; u < CG; ++u) pd[u] = 0.0;
        for (int i = o + 1 + ln; i < o + d; i += 64) {
          const double wb = LV(WB + i);
#pragma unroll
          for (int u = 0; u < CG; ++u) pd[u] = fma(wb, GC(u, i), pd[u]);
        }
        const double im = ccv(CC_IMU, c), wb0 = ccv(CC_WB0, c), i1 = ccv(CC_I1, c);
        double cst[CG];
#pragma unroll
        for (int u = 0; u < CG; ++u) {
          const double del = wave_sum(pd[u]);
          const double gh = GC(u, o);
          cst[u] = -gh + del * i1;
          if (ln == 0) x0[u * KP + o] = (u < nl) ? im * (wb0 * gh - del) : 0.0;
        }
        for (int i = o + 1 + ln; i < o + d; i += 64) {
          const double wb = LV(WB + i);
#pragma unroll
          for (int u = 0; u < CG; ++u) x0[u * KP + i] = (u < nl) ? im * (GC(u, i) + cst[u] * wb) : 0.0;
        }
      }
#undef GC
      for (int i = kk + ln; i < KP; i += 64) {
#pragma unroll
        for (int u = 0; u < CG; ++u) x0[u * KP + i] = 0.0;
      }
    }
    BAR();
  }

  // ------------------------------------------------ staged SYRK (LDS-DMA)
  // H = X'X with X streamed through LDS in 4-row chunks (all NPAD columns,
  // 32 contiguous bytes per column), shared by the eight wavefronts: each
  // wavefront accumulates one 64x64 block per pass over X (ceil(blocks / 8)
  // passes), so X is read once per pass instead of two 64-column panels per
  // block.  The chunks land in LDS by global_load_lds_dwordx4 (no VGPRs: the
  // kernel is at the 256-VGPR cap of 8 waves per CU), three chunks in flight
  // in a ring of four buffers; one LDS barrier per chunk, preceded by a
  // counted vmcnt that retires this wave's DMA of the chunk about to be read
  // (its DMAs of the two younger chunks stay in flight).  The asm DMAs are
  // outside hipcc's wait bookkeeping; extra in-flight ops only strengthen the
  // waits it emits for its own loads.
#ifndef SOCP_LG_STAGED
#define SOCP_LG_STAGED 0  // A/B: 1 = the LDS-DMA staged SYRK
#endif
  // a 64-bit pointer made wave-uniform (SGPRs): __builtin_amdgcn_readfirstlane
  // takes and returns int, so the halves go separately
  __device__ __forceinline__ static gcdbl* uni_ptr(gcdbl* p) {
    const unsigned long long v = (unsigned long long)p;
    const unsigned lo = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)v);
    const unsigned hi = (unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(v >> 32));
    return (gcdbl*)(((unsigned long long)hi << 32) | lo);
  }
  template <int N>
  __device__ __forceinline__ static void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
  }
  // this wave's DMA of chunk c: column groups cg = w + 8t (t < GPW) of 32
  // columns; lane L copies rows 4c + 2(L & 1) .. +1 of column 32 cg + L/2 to
  // byte 1024 cg + 16 L of the buffer (lane-linear)
  // (saddr form: X's base in SGPRs, a 32-bit per-lane byte offset)
  // base: the chunk's first row of column 0 (wave-uniform); voff[t]: the
  // lane's byte offset from it (loop-invariant)
  template <int GPW>
  __device__ __forceinline__ static void glds_chunk(gcdbl* base, const unsigned (&voff)[GPW], unsigned bufb, int w) {
#pragma unroll
    for (int t = 0; t < GPW; ++t) {
      const unsigned dst = __builtin_amdgcn_readfirstlane(bufb + 1024u * (unsigned)(w + 8 * t));
      unsigned keep;
      asm volatile(
          "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
          : "=&s"(keep)
          : "v"(voff[t]), "s"(base), "s"(dst)
          : "memory");
    }
  }
  // noinline: its own register allocation (the kernel body is at the 256-VGPR
  // cap and spills; a scratch reload inside the chunk loop would wait for every
  // DMA in flight)
  template <int GPW>
  __device__ __attribute__((noinline)) void form_H_staged_g(bool addAA) {
#define UNI(x) __builtin_amdgcn_readfirstlane(x)
    const int NP = UNI(L.NPAD), KP = UNI(L.KP), NB = NP / 64, nblk = NB * (NB + 1) / 2, NCH = KP / 4;
    const int w_ = UNI(wv), b0 = UNI(L.o_kvd);
#undef UNI
    const int ln = lane, g = lane >> 4, cl = lane & 15;
    gcdbl* const xw = uni_ptr((gcdbl*)Xw);
    // buffer q: LDS double offset and byte address (arithmetic, not a local
    // array: a dynamically indexed array would live in scratch)
    const int CS = 4 * NP;
    const unsigned lbase = (unsigned)(uintptr_t)((__attribute__((address_space(3))) double*)lg_lds);
    auto boff = [&](int q) { return b0 + q * CS; };
    auto bbyte = [&](int q) { return lbase + 8u * (unsigned)boff(q); };
    // A'A (sing) rides along as the rows of A after those of X: [X; A]'[X; A]
    gcdbl* const ap = uni_ptr((gcdbl*)Ap);
    const int MP = __builtin_amdgcn_readfirstlane(L.MPAD);
    const int NCT = __builtin_amdgcn_readfirstlane(NCH + (addAA ? MP / 4 : 0));
    // lane L of column group cg copies 16 bytes: column 32 cg + L/2, rows 2(L & 1) .. +1
    // X is chunk-major (form_X_fast(chunked)): a wave-instruction copies 1 KiB
    // of contiguous bytes; A (column-major, leading dimension MPAD) 32 bytes per column
    unsigned vx[GPW], va[GPW];
#pragma unroll
    for (int t = 0; t < GPW; ++t) {
      const int col = 32 * (w_ + 8 * t) + (ln >> 1);
      vx[t] = (unsigned)((128 * (w_ + 8 * t) + 2 * ln) * 8);
      va[t] = (unsigned)((col * MP + 2 * (ln & 1)) * 8);
    }
    auto issue = [&](int c) {
      if (c < NCH)
        glds_chunk<GPW>(xw + (int64_t)4 * NP * c, vx, bbyte(c & 3), w_);
      else
        glds_chunk<GPW>(ap + 4 * (c - NCH), va, bbyte(c & 3), w_);
    };
    for (int pass = 0; pass * NW < nblk; ++pass) {
      const int b = pass * NW + w_;
      const bool act = b < nblk;
      int I = 0, J = 0;
      if (act) tri_ij(b, I, J);
      I = __builtin_amdgcn_readfirstlane(I);
      J = __builtin_amdgcn_readfirstlane(J);
      const bool dg = I == J;
      d4 acc[4][4];
      zero_blk(acc);
      // vmcnt(0) as the builtin (hipcc tracks it): the previous pass's block
      // stores retire here, not in every chunk step (with them pending at the
      // loop head, hipcc waits vmcnt(0) before each step's LDS reads, which
      // would also drain the DMA ring)
      __builtin_amdgcn_s_waitcnt(0x0F70);
#pragma unroll
      for (int q = 0; q < 3; ++q)
        if (q < NCT) issue(q);
      for (int c = 0; c < NCT; ++c) {
        const int ahead = NCT - 1 - c;  // chunks issued after c (at most 2 at this point)
        if (ahead >= 2)
          wait_vm<2 * GPW>();
        else if (ahead == 1)
          wait_vm<GPW>();
        else
          wait_vm<0>();
        LDS_BAR();
        if (c + 3 < NCT) issue(c + 3);
        if (act) {  // all 16 tiles, also on a diagonal block (one code path: a
                    // branch between tile sets costs register copies of acc)
          const int buf = boff(c & 3);
          double av[4], bv[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            av[t] = LV(buf + (64 * I + 16 * t + cl) * 4 + g);
            bv[t] = LV(buf + (64 * J + 16 * t + cl) * 4 + g);
          }
#pragma unroll
          for (int ta = 0; ta < 4; ++ta)
#pragma unroll
            for (int tb = 0; tb < 4; ++tb) acc[ta][tb] = mfma(av[ta], bv[tb], acc[ta][tb]);
        }
      }
      if (act) {
        if (dg)
          store_blk<true>(acc, Hm, NP, 64 * I, 64 * J, n);
        else
          store_blk(acc, Hm, NP, 64 * I, 64 * J, n);
      }
      LDS_BAR();  // every read of this pass done before the next pass restages
    }
    // the buffers overlay the dead k-vectors: zero them again (their padding
    // rows must read 0)
    for (int e = tid; e < 7 * KP; e += NTH) LV(b0 + e) = 0.0;
    BAR();
  }
  // the LDS-DMA destination (M0) kept inside the first 64 KiB
  __device__ bool staged_ok() const {
    if constexpr (GV) return false;  // the staged SYRK's buffers are LDS
    const unsigned lbase = (unsigned)(uintptr_t)((__attribute__((address_space(3))) double*)(lg_lds + L.o_kvd));
    return SOCP_LG_STAGED && L.sy && lbase + 128u * (unsigned)L.NPAD <= 65536u;
  }
  __device__ void form_H_staged(bool addAA) {
    if (L.NPAD == 512)
      form_H_staged_g<2>(addAA);
    else
      form_H_staged_g<1>(addAA);
  }

  // H = X'X (+A'A) (densesolver.jl:42-46): lower 64x64 blocks, one wavefront
  // per block; padding diagonal = 1.
  __device__ __forceinline__ static int syrk_order8(int t) {
    // (I << 3) | J of the t-th block, rounds of eight (form_H)
#if SOCP_LG_SYRK_ORDER == 2
    // also balanced over the SIMDs (wavefronts w and w + 4 share one): the
    // diagonal blocks (10 of 16 tiles) of rounds 1 and 2 on wavefronts 0-3
    // beside an off-diagonal block each, the last round's four blocks on
    // wavefronts 0-3 -- every SIMD issues the same MFMAs between barriers
    // (132 tile-steps per k-step in all, the 528 / 4 minimum; 26 panel reads)
    constexpr unsigned char tab[36] = {
        0x00, 0x09, 0x12, 0x1b, 0x08, 0x10, 0x11, 0x18,  // panels 0..3: diagonal, off-diagonal
        0x24, 0x2d, 0x36, 0x3f, 0x2c, 0x34, 0x35, 0x3c,  // panels 4..7
        0x20, 0x21, 0x22, 0x23, 0x28, 0x29, 0x2a, 0x2b,  // {4,5} x {0..3}
        0x30, 0x31, 0x32, 0x33, 0x38, 0x39, 0x3a, 0x3b,  // {6,7} x {0..3}
        0x19, 0x1a, 0x3d, 0x3e};                         // (3,1) (3,2) (7,5) (7,6)
#else
    constexpr unsigned char tab[36] = {
        0x00, 0x08, 0x09, 0x10, 0x11, 0x12, 0x18, 0x19,  // panels 0..3
        0x24, 0x2c, 0x2d, 0x34, 0x35, 0x36, 0x3c, 0x3d,  // panels 4..7
        0x20, 0x21, 0x22, 0x23, 0x28, 0x29, 0x2a, 0x2b,  // {4,5} x {0..3}
        0x30, 0x31, 0x32, 0x33, 0x38, 0x39, 0x3a, 0x3b,  // {6,7} x {0..3}
        0x1a, 0x1b, 0x3e, 0x3f};                         // (3,2) (3,3) (7,6) (7,7)
#endif
    return tab[t];
  }
  __device__ void form_H(bool addAA) {
    const int NB = L.NPAD / 64, nblk = NB * (NB + 1) / 2;
#if SOCP_LG_SYRK_SYNC > 0
    // The eight wavefronts' blocks of one round share X panels (row-major
    // lower triangle: round 1 reads panels 0..3 for 8 blocks), but a panel
    // row is in L2 only while the wavefronts are within a few k-steps of one
    // another.  A workgroup barrier every SOCP_LG_SYRK_SYNC rows of k keeps
    // them in step, so a round reads each of its panels from HBM once instead
    // of once per block.  Idle wavefronts of the last round keep the count.
    if (!addAA) {
      constexpr int KB = SOCP_LG_SYRK_SYNC;
      const int KP = L.KP;
      for (int r = 0; r < nblk; r += NW) {
        const int t = r + wv;
        int I = 0, J = 0;
        if (t < nblk) {
          if (SOCP_LG_SYRK_ORDER && NB == 8 && NW == 8) {
            // rounds over few panels: the 0..3 and 4..7 triangles (4 panels
            // each), {4,5} x {0..3} and {6,7} x {0..3} (6 each), the rest (4):
            // 24 panel reads per SYRK instead of the row-major order's 30
            const int code = syrk_order8(t);
            I = code >> 3;
            J = code & 7;
          } else {
            tri_ij(t, I, J);
          }
        }
        d4 acc[4][4];
        zero_blk(acc);
        for (int k0 = 0; k0 < KP; k0 += KB) {
          const int kr = KP - k0 < KB ? KP - k0 : KB;
          if (t < nblk) {
            if (I == J)
              blk_gemm<true>(acc, Xw + k0, Xw + k0, KP, 64 * I, 64 * J, kr, true, -1);
            else
              blk_gemm(acc, Xw + k0, Xw + k0, KP, 64 * I, 64 * J, kr, false, -1);
          }
          __builtin_amdgcn_s_barrier();
        }
        if (t < nblk) {
          if (I == J)
            store_blk<true>(acc, Hm, L.NPAD, 64 * I, 64 * J, n);
          else
            store_blk(acc, Hm, L.NPAD, 64 * I, 64 * J, n);
        }
      }
      BAR();
      return;
    }
#endif
    for (int t = wv; t < nblk; t += NW) {
      int I, J;
      tri_ij(t, I, J);
      d4 acc[4][4];
      zero_blk(acc);
      if (I == J) {  // diagonal block: only the tiles on and below the diagonal
        blk_gemm<true>(acc, Xw, Xw, L.KP, 64 * I, 64 * J, L.KP, true, -1);
        if (addAA) blk_gemm<true>(acc, Ap, Ap, L.MPAD, 64 * I, 64 * J, L.MPAD, true, -1);
        store_blk<true>(acc, Hm, L.NPAD, 64 * I, 64 * J, n);
      } else {
        blk_gemm(acc, Xw, Xw, L.KP, 64 * I, 64 * J, L.KP, false, -1);
        if (addAA) blk_gemm(acc, Ap, Ap, L.MPAD, 64 * I, 64 * J, L.MPAD, false, -1);
        store_blk(acc, Hm, L.NPAD, 64 * I, 64 * J, n);
      }
    }
    BAR();
  }

  // One panel of the sweep below by 16x16 tiles on MFMA: the 64 rank-1 pivot
  // steps regrouped into a tile Cholesky of the pivot block.  With D = M_PP =
  // L L' (tile rows t = 0..3 of the panel; W_t = L_tt^-1 by factor_tile, whose
  // 4x4 pivots are D's Cholesky pivots: the same potrf failure test):
  //   forward  Y_t = W_t (R_t - sum_{s<t} L_ts Y_s), L_ts = Y(s, P-tile t)'
  //            -- Y = L^-1 M_P, the rows the Gram updates read (fv = -1);
  //            in the P block Y = L', whose lower tiles are replaced by
  //            E = L^-1 (the identity's forward pass);
  //   backward Z_t = W_t' (Y_t - sum_{u>t} L_ut' Z_u)
  //            -- Z = D^-1 M_P off the P block, D^-1 = L'^-1 E in it;
  //   M_P <- Z, M_PP <- -D^-1 (its lower triangle, from one tile of each
  //   mirrored pair: every element has one writer).
  // Wave w holds tile columns j = w + 8i of the panel's four tile rows; each
  // of the 4 + 4 steps publishes the tiles the others need through four LDS
  // tile slots at o_row (8 LDS barriers per panel instead of 64 pivot steps).
  // CHOL: the Cholesky factorisation's panel instead (chol_nb): the columns
  // left of the panel are not touched, and after the forward pass the panel
  // is stored in place -- Y = L_PP^-1 M_P,J = L_JP' (J > P) as columns of L,
  // and E = L_PP^-1 in the diagonal block (lower triangle, column-major).
  template <int nb, bool CHOL = false>
  __device__ __forceinline__ bool panel_tiles(gdbl* M, int ld, int P) {
    constexpr int NT = 4 * nb, NJ = (NT + NW - 1) / NW;
    const int w = wv, RW = L.RW, P0 = 64 * P, ob = L.o_row, of = L.o_rv;
    gdbl* const Y = Yp + (int64_t)P * 64 * RW;
    const d4 zero = {0.0, 0.0, 0.0, 0.0};
    d4 R[4][NJ];
    {
      LANE_IDS();
#pragma unroll
      for (int i = 0; i < NJ; ++i) {
        const int j = w + NW * i;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int x = P0 + 16 * t + g + 4 * r, y = 16 * j + cl;  // element (x, y), lower triangle
            R[t][i][r] = (j < NT && (!CHOL || j >= 4 * P)) ? M[(y <= x) ? (int64_t)y * ld + x : (int64_t)x * ld + y] : 0.0;
          }
      }
    }
    // ---- forward pass
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      LANE_IDS();
      const int jd = 4 * P + t, od = jd % NW, id = jd / NW;
      if (w == od) {
        d4 C = zero, Ys[4];
#pragma unroll
        for (int i = 0; i < NJ; ++i)
          if (i == id) {
            C = R[t][i];
#pragma unroll
            for (int s_ = 0; s_ < t; ++s_) Ys[s_] = R[s_][i];
          }
#pragma unroll
        for (int s_ = 0; s_ < t; ++s_) C = tile_mm<1>(Ys[s_], Ys[s_], C);  // D_tt - sum L_ts L_ts'
        d4 Wt;
        bool ok = true;
        factor_tile<SOCP_LG_TILE_INPLACE != 0>(C, Wt, ok);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
#pragma unroll
          for (int s_ = 0; s_ < t; ++s_) LV(ob + 256 * s_ + 64 * r + lane) = Ys[s_][r];
          LV(ob + 768 + 64 * r + lane) = Wt[r];
        }
        if (lane == 0) LV(of + t) = ok ? 0.0 : 1.0;
#pragma unroll
        for (int i = 0; i < NJ; ++i)
          if (i == id) R[t][i] = Wt;  // E's diagonal tile
      }
      LDS_BAR();
      d4 Yb[4], WT;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int s_ = 0; s_ < t; ++s_) Yb[s_][r] = LV(ob + 256 * s_ + 64 * r + lane);
        WT[r] = LV(ob + 768 + 64 * (cl >> 2) + 16 * (cl & 3) + g + 4 * r);  // W_t'
      }
#pragma unroll
      for (int i = 0; i < NJ; ++i) {
        const int j = w + NW * i;
        if (j >= NT || j == jd || (CHOL && j < 4 * P)) continue;
        const int u = ((j >> 2) == P) ? (j & 3) : -1;  // P-block tile column index
        d4 X = (u >= 0 && u < t) ? zero : R[t][i];      // E: the identity's zero below
#pragma unroll
        for (int s_ = 0; s_ < t; ++s_)
          if (u < 0 || u >= t || s_ >= u) X = tile_mm<1>(Yb[s_], R[s_][i], X);
        R[t][i] = tile_mm<0>(WT, X, zero);
      }
      LDS_BAR();
    }
    bool ok = true;
#pragma unroll
    for (int t = 0; t < 4; ++t) ok = ok && LV(of + t) == 0.0;
    if (!ok) return false;  // uniform: every wave read the same flags
    if constexpr (CHOL) {
      LANE_IDS();
#pragma unroll
      for (int i = 0; i < NJ; ++i) {
        const int j = w + NW * i;
        if (j >= NT || j < 4 * P) continue;
        const bool pb = (j >> 2) == P;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int x = P0 + 16 * t + g + 4 * r, y = 16 * j + cl;  // tile element (x, y)
            if (!pb)
              M[(int64_t)x * ld + y] = R[t][i][r];  // L[y][x]: column x of L, coalesced
            else if ((j & 3) <= t && y <= x)
              M[(int64_t)y * ld + x] = R[t][i][r];  // E[x][y]
          }
      }
      if (tid < 64) Rv[P0 + tid] = -1.0;
      return true;
    }
    {
      // the Gram updates' rows: Y off the P block, and fv = -1 (rows are L^-1-scaled)
      LANE_IDS();
#pragma unroll
      for (int i = 0; i < NJ; ++i) {
        const int j = w + NW * i;
        if (j >= NT || (j >> 2) == P) continue;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) Y[(int64_t)(16 * t + g + 4 * r) * RW + 16 * j + cl] = R[t][i][r];
      }
      if (tid < 64) Rv[P0 + tid] = -1.0;
    }
    // ---- backward pass
#pragma unroll
    for (int t = 3; t >= 0; --t) {
      LANE_IDS();
#pragma unroll
      for (int u = t; u < 4; ++u) {
        const int jj = 4 * P + u;
        if (w == jj % NW) {
#pragma unroll
          for (int i = 0; i < NJ; ++i)
            if (i == jj / NW) {
#pragma unroll
              for (int r = 0; r < 4; ++r) LV(ob + 256 * u + 64 * r + lane) = R[t][i][r];  // W_t, Y(t, P-tile u)
            }
        }
      }
      LDS_BAR();
      d4 Wt, YT[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        Wt[r] = LV(ob + 256 * t + 64 * r + lane);
#pragma unroll
        for (int u = t + 1; u < 4; ++u) YT[u][r] = LV(ob + 256 * u + 64 * (cl >> 2) + 16 * (cl & 3) + g + 4 * r);
      }
#pragma unroll
      for (int i = 0; i < NJ; ++i) {
        const int j = w + NW * i;
        if (j >= NT) continue;
        const int v = ((j >> 2) == P) ? (j & 3) : -1;
        d4 X = (v > t) ? zero : R[t][i];  // in the P block: E (zero above its diagonal)
#pragma unroll
        for (int u = t + 1; u < 4; ++u) X = tile_mm<1>(YT[u], R[u][i], X);
        R[t][i] = tile_mm<0>(Wt, X, zero);
      }
      LDS_BAR();
    }
    {
      LANE_IDS();
#pragma unroll
      for (int i = 0; i < NJ; ++i) {
        const int j = w + NW * i;
        if (j >= NT) continue;
        const bool pb = (j >> 2) == P;
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int x = P0 + 16 * t + g + 4 * r, y = 16 * j + cl;
            if (pb) {
              if (y <= x) M[(int64_t)y * ld + x] = -R[t][i][r];
            } else {
              M[(y <= x) ? (int64_t)y * ld + x : (int64_t)x * ld + y] = R[t][i][r];
            }
          }
      }
    }
    return true;
  }

  // In-place blocked Cholesky H = L L' (densesolver.jl:47 cholesky!; the
  // explicit Li = H^-1 of :48 is never formed, its products are triangular
  // solves against L -- see solve_matrix_part).  Left-looking by 64-column
  // panels: block (t, P), t >= P, first receives the Gram updates of the
  // panels Q < P (its columns of L read as rows: column x of L is contiguous),
  // then panel_tiles<CHOL> factors the pivot block by 16x16 tiles and stores
  // L_JP and E_P = L_PP^-1.  A pivot <= 0 or NaN fails as potrf does.
  template <int nb>
  __device__ bool chol_nb(gdbl* M, int ld) {
    for (int P = 0; P < nb; ++P) {
      if (P > 0 && SOCP_LG_CATCH_SPLIT && SOCP_LG_CATCH_SPLIT_K * (nb - P) <= NW) {
        // few blocks left: each block's catch-up split into its four 16-column
        // groups, one per wavefront (bitwise the whole-block result)
        for (int it = wv; it < 4 * (nb - P); it += NW) {
          const int t = P + it / 4, a_ = it % 4;
          d4 acc[4];
          if (t == P) {
            load_colT<true>(acc, M, ld, 64 * t, 64 * P, a_);
            for (int Q = 0; Q < P; ++Q) gram_colT<true>(acc, M + (int64_t)64 * Q * ld, ld, 64 * t, 64 * P, Rv + 64 * Q, a_);
            store_colT<true>(acc, M, ld, 64 * t, 64 * P, a_);
          } else {
            load_colT(acc, M, ld, 64 * t, 64 * P, a_);
            for (int Q = 0; Q < P; ++Q) gram_colT(acc, M + (int64_t)64 * Q * ld, ld, 64 * t, 64 * P, Rv + 64 * Q, a_);
            store_colT(acc, M, ld, 64 * t, 64 * P, a_);
          }
        }
        BAR();
      } else if (P > 0) {
        for (int t = P + wv; t < nb; t += NW) {
          d4 acc[4][4];
          if (t == P) {
            load_blkT<true>(acc, M, ld, 64 * t, 64 * P);
            for (int Q = 0; Q < P; ++Q) gram_blkT<true>(acc, M + (int64_t)64 * Q * ld, ld, 64 * t, 64 * P, Rv + 64 * Q);
            store_blkT<true>(acc, M, ld, 64 * t, 64 * P);
          } else {
            load_blkT(acc, M, ld, 64 * t, 64 * P);
            for (int Q = 0; Q < P; ++Q) gram_blkT(acc, M + (int64_t)64 * Q * ld, ld, 64 * t, 64 * P, Rv + 64 * Q);
            store_blkT(acc, M, ld, 64 * t, 64 * P);
          }
        }
        BAR();
      }
      LSTAMP(NSTAMP + 1 + 0);
      const bool ok = panel_tiles<nb, true>(M, ld, P);
      LSTAMP(NSTAMP + 1 + 1);
      if (!ok) return false;
      BAR();  // L's panel P complete before the next catch-up reads it
      LSTAMP(NSTAMP + 1 + 2);
    }
    return true;
  }
  // CHOL panels wider than panel_tiles' register window (NPAD > 512: more than
  // 32 tile columns right of the panel's block).  The window of WT tile columns
  // starting at the P block runs panel_tiles' forward pass (the four tile
  // factorisations); the tiles each step publishes -- Y_s (s < t) and W_t' --
  // are also saved to the workspace (Yp: unused while chol runs), and each
  // later window of WT tile columns replays the four steps with them.  Every
  // tile gets the operations panel_tiles would apply, in the same order, so the
  // factor does not depend on the window.  Stores as panel_tiles<CHOL>.
  static constexpr int WJ = 4, WTC = WJ * NW;  // tile columns per wave / per window
  __device__ bool panel_chol_wide(gdbl* M, int ld, int P, int NT) {
    const int w = wv, P0 = 64 * P, ob = L.o_row, of = L.o_rv, J0 = 4 * P;
    gdbl* const sv = Yp;  // step t's tiles: slot 4t + s (Y_s, s < t), 4t + 3 (W_t'), lane order
    const d4 zero = {0.0, 0.0, 0.0, 0.0};
    for (int jw = J0; jw < NT; jw += WTC) {
      const bool first = jw == J0;
      d4 R[4][WJ];
      {
        LANE_IDS();
#pragma unroll
        for (int i = 0; i < WJ; ++i) {
          const int j = jw + w + NW * i;
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int x = P0 + 16 * t + g + 4 * r, y = 16 * j + cl;  // element (x, y), lower triangle
              R[t][i][r] = j < NT ? M[(y <= x) ? (int64_t)y * ld + x : (int64_t)x * ld + y] : 0.0;
            }
        }
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        LANE_IDS();
        const int jd = J0 + t;  // in the first window: wave t, register column 0
        d4 Yb[4], WTt;
        if (first) {
          if (w == t) {
            d4 C = R[t][0], Ys[4];
#pragma unroll
            for (int s_ = 0; s_ < t; ++s_) Ys[s_] = R[s_][0];
#pragma unroll
            for (int s_ = 0; s_ < t; ++s_) C = tile_mm<1>(Ys[s_], Ys[s_], C);  // D_tt - sum L_ts L_ts'
            d4 Wt;
            bool ok = true;
            factor_tile<SOCP_LG_TILE_INPLACE != 0>(C, Wt, ok);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
#pragma unroll
              for (int s_ = 0; s_ < t; ++s_) LV(ob + 256 * s_ + 64 * r + lane) = Ys[s_][r];
              LV(ob + 768 + 64 * r + lane) = Wt[r];
            }
            if (lane == 0) LV(of + t) = ok ? 0.0 : 1.0;
            R[t][0] = Wt;  // E's diagonal tile
          }
          LDS_BAR();
#pragma unroll
          for (int r = 0; r < 4; ++r) {
#pragma unroll
            for (int s_ = 0; s_ < t; ++s_) Yb[s_][r] = LV(ob + 256 * s_ + 64 * r + lane);
            WTt[r] = LV(ob + 768 + 64 * (cl >> 2) + 16 * (cl & 3) + g + 4 * r);  // W_t'
          }
          if (w == 0) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
#pragma unroll
              for (int s_ = 0; s_ < t; ++s_) sv[(4 * t + s_) * 256 + 64 * r + lane] = Yb[s_][r];
              sv[(4 * t + 3) * 256 + 64 * r + lane] = WTt[r];
            }
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
#pragma unroll
            for (int s_ = 0; s_ < t; ++s_) Yb[s_][r] = sv[(4 * t + s_) * 256 + 64 * r + lane];
            WTt[r] = sv[(4 * t + 3) * 256 + 64 * r + lane];
          }
        }
#pragma unroll
        for (int i = 0; i < WJ; ++i) {
          const int j = jw + w + NW * i;
          if (j >= NT || j == jd) continue;
          const int u = ((j >> 2) == P) ? (j & 3) : -1;  // P-block tile column index
          d4 X = (u >= 0 && u < t) ? zero : R[t][i];      // E: the identity's zero below
#pragma unroll
          for (int s_ = 0; s_ < t; ++s_)
            if (u < 0 || u >= t || s_ >= u) X = tile_mm<1>(Yb[s_], R[s_][i], X);
          R[t][i] = tile_mm<0>(WTt, X, zero);
        }
        if (first) LDS_BAR();  // the slots are rewritten by the next step
      }
      if (first) {
        bool ok = true;
#pragma unroll
        for (int t = 0; t < 4; ++t) ok = ok && LV(of + t) == 0.0;
        if (!ok) return false;  // uniform: every wave read the same flags
      }
      {
        LANE_IDS();
#pragma unroll
        for (int i = 0; i < WJ; ++i) {
          const int j = jw + w + NW * i;
          if (j >= NT) continue;
          const bool pb = (j >> 2) == P;
#pragma unroll
          for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int x = P0 + 16 * t + g + 4 * r, y = 16 * j + cl;  // tile element (x, y)
              if (!pb)
                M[(int64_t)x * ld + y] = R[t][i][r];  // L[y][x]: column x of L, coalesced
              else if ((j & 3) <= t && y <= x)
                M[(int64_t)y * ld + x] = R[t][i][r];  // E[x][y]
            }
        }
      }
      if (first) BAR();  // the saved step tiles visible to every wave
    }
    if (tid < 64) Rv[P0 + tid] = -1.0;
    return true;
  }
  // chol_nb with a runtime panel count and panel_chol_wide (NPAD > 512)
  __device__ bool chol_wide(gdbl* M, int ld) {
    const int nb = ld / 64;
    for (int P = 0; P < nb; ++P) {
      if (P > 0) {
        for (int t = P + wv; t < nb; t += NW) {
          d4 acc[4][4];
          if (t == P) {
            load_blkT<true>(acc, M, ld, 64 * t, 64 * P);
            for (int Q = 0; Q < P; ++Q) gram_blkT<true>(acc, M + (int64_t)64 * Q * ld, ld, 64 * t, 64 * P, Rv + 64 * Q);
            store_blkT<true>(acc, M, ld, 64 * t, 64 * P);
          } else {
            load_blkT(acc, M, ld, 64 * t, 64 * P);
            for (int Q = 0; Q < P; ++Q) gram_blkT(acc, M + (int64_t)64 * Q * ld, ld, 64 * t, 64 * P, Rv + 64 * Q);
            store_blkT(acc, M, ld, 64 * t, 64 * P);
          }
        }
        BAR();
      }
      const bool ok = panel_chol_wide(M, ld, P, 4 * nb);
      if (!ok) return false;
      BAR();  // L's panel P complete before the next catch-up reads it
    }
    return true;
  }
  __device__ bool chol(gdbl* M, int ld) {
    if (ld > 64 * LARGE_NB_MAX) return chol_wide(M, ld);
    switch (ld / 64) {
      case 1: return chol_nb<1>(M, ld);
      case 2: return chol_nb<2>(M, ld);
      case 3: return chol_nb<3>(M, ld);
      case 4: return chol_nb<4>(M, ld);
      case 5: return chol_nb<5>(M, ld);
      case 6: return chol_nb<6>(M, ld);
      case 7: return chol_nb<7>(M, ld);
      default: return chol_nb<8>(M, ld);
    }
  }

  // Z = L^-1 A' (NPAD x MPAD, row-major in Tm) by block forward substitution:
  // Z_P = E_P (A'_P - sum_{y < 64P} L[P rows][y] Z[y]), 16x16 output tiles
  // dealt over the wavefronts (MFMA: A operand = L / E read down a column,
  // B operand = rows of Z); R = A'_P - ... is staged in Yp (row-major 64 x
  // MPAD) between the two products.
  __device__ void chol_fwd_multi(gcdbl* Lm, int ld) {
    const int NB = L.NPAD / 64, MT = L.MPAD / 16, MP = L.MPAD;
    gdbl* const Rs = Yp;
    const d4 zero = {0.0, 0.0, 0.0, 0.0};
    for (int P = 0; P < NB; ++P) {
      const int P0 = 64 * P;
      for (int tt = wv; tt < 4 * MT; tt += NW) {
        LANE_IDS();
        const int ta = tt / MT, tb = tt - ta * MT;
        d4 acc0, acc1 = zero;
#pragma unroll
        for (int r = 0; r < 4; ++r) acc0[r] = Ap[(int64_t)(P0 + 16 * ta + g + 4 * r) * MP + 16 * tb + cl];
        // 4 SOCP_LG_ZU rows per round, their loads issued before the MFMAs (one
        // memory round trip per 32 rows instead of per 8); acc0 / acc1 take the
        // same rows in the same order as before
        for (int y0 = 0; y0 < P0; y0 += 4 * SOCP_LG_ZU) {
          double a[SOCP_LG_ZU], b[SOCP_LG_ZU];
#pragma unroll
          for (int u = 0; u < SOCP_LG_ZU; ++u) {
            a[u] = Lm[(int64_t)(y0 + 4 * u + g) * ld + P0 + 16 * ta + cl];
            b[u] = Tm[(int64_t)(y0 + 4 * u + g) * MP + 16 * tb + cl];
          }
#pragma unroll
          for (int u = 0; u < SOCP_LG_ZU; u += 2) {
            acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u], b[u], acc0, 0, 0, 1);  // -= L Z
            acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u + 1], b[u + 1], acc1, 0, 0, 1);
          }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) Rs[(int64_t)(16 * ta + g + 4 * r) * MP + 16 * tb + cl] = acc0[r] + acc1[r];
      }
      BAR();
      for (int tt = wv; tt < 4 * MT; tt += NW) {
        LANE_IDS();
        const int ta = tt / MT, tb = tt - ta * MT, i = 16 * ta + cl;
        d4 acc = zero;
        for (int x0 = 0; x0 <= 16 * ta + 12; x0 += 16) {  // E is lower: x <= i; 4 steps per round trip
          double av[4], bv[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const int x = x0 + 4 * u + g;
            av[u] = (x <= i) ? Lm[(int64_t)(P0 + x) * ld + P0 + i] : 0.0;
            bv[u] = Rs[(int64_t)x * MP + 16 * tb + cl];
          }
#pragma unroll
          for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], bv[u], acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) Tm[(int64_t)(P0 + 16 * ta + g + 4 * r) * MP + 16 * tb + cl] = acc[r];
      }
      BAR();
    }
  }

  // S = Z'Z = A Li A' (lower 64x64 blocks; the padded diagonal gets the
  // identity, as store_blk's)
  __device__ void form_S_gram() {
    const int NB = L.NPAD / 64, MB = L.MPAD / 64, MP = L.MPAD;
    for (int t = wv; t < MB * (MB + 1) / 2; t += NW) {
      LANE_IDS();
      int I, J;
      tri_ij(t, I, J);
      d4 acc[4][4];
      zero_blk(acc);
      for (int P = 0; P < NB; ++P) {
        if (I == J)
          gram_blkT<true, false>(acc, Tm + (int64_t)64 * P * MP, MP, 64 * I, 64 * J, nullptr);
        else
          gram_blkT<false, false>(acc, Tm + (int64_t)64 * P * MP, MP, 64 * I, 64 * J, nullptr);
      }
      if (I == J) {
#pragma unroll
        for (int a_ = 0; a_ < 4; ++a_)
#pragma unroll
          for (int b_ = 0; b_ < 4; ++b_)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = 64 * I + 16 * b_ + cl, col = 64 * J + 16 * a_ + g + 4 * r;
              if (row == col && row >= m) acc[a_][b_][r] = 1.0;
            }
        store_blkT<true>(acc, Sm, MP, 64 * I, 64 * J);
      } else {
        store_blkT(acc, Sm, MP, 64 * I, 64 * J);
      }
    }
    BAR();
  }

  // The explicit inverse from the factor chol() leaves in M (column-major, L
  // below the diagonal blocks, E_P = L_PP^-1 in them): densesolver.jl:47-48,
  // Li = ldiv!(cholesky!(H), I) = L^-T L^-1.
  // (1) Y = L^-1 (row-major in Yp, ld x ld) by block forward substitution, one
  //     64-row panel per step: a wavefront owns a 16-column tile of the panel
  //     rows, R = -sum_{c0 <= y < P0} L[P rows][y] Y[y][cols] (four 16x16
  //     accumulators, MFMA, Y lower so the sum starts at the tile's column),
  //     then Y[P rows][cols] = E_P R; the diagonal block is E_P itself;
  // (2) M = Y'Y in both triangles (64x64 blocks, the Gram products of the
  //     panels P >= I of block (I, J), as form_S_gram), symmetric by
  //     construction.  Padding rows / columns carry the identity through.
  __device__ void chol_inverse(gdbl* M, int ld) {
    const int NB = ld / 64;
    gdbl* const Y = Yp;
    const d4 zero = {0.0, 0.0, 0.0, 0.0};
    for (int P = 0; P < NB; ++P) {
      const int P0 = 64 * P;
      for (int tb = wv; tb < 4 * P + 4; tb += NW) {
        LANE_IDS();
        const int c0 = 16 * tb;
        d4 out[4];
        if (tb >= 4 * P) {
          const int x = c0 - P0 + cl;  // E_P lower: zero above its diagonal
#pragma unroll
          for (int ta = 0; ta < 4; ++ta)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int i = 16 * ta + g + 4 * r;
              out[ta][r] = (x <= i) ? M[(int64_t)(P0 + x) * ld + P0 + i] : 0.0;
            }
        } else {
          d4 acc[4] = {zero, zero, zero, zero};
          for (int y0 = c0; y0 < P0; y0 += 16) {  // 16 rows per round trip
            double a[4][4], b[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int y = y0 + 4 * u + g;
              b[u] = Y[(int64_t)y * ld + c0 + cl];
#pragma unroll
              for (int ta = 0; ta < 4; ++ta) a[u][ta] = M[(int64_t)y * ld + P0 + 16 * ta + cl];
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
              for (int ta = 0; ta < 4; ++ta)
                acc[ta] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[u][ta], b[u], acc[ta], 0, 0, 1);  // -= L Y
          }
#pragma unroll
          for (int tc = 0; tc < 4; ++tc) {  // out_tc = sum_{ta <= tc} E[tc][ta] R_ta
            d4 o = zero;
#pragma unroll
            for (int ta = 0; ta <= tc; ++ta)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int x = 16 * ta + g + 4 * r, i = 16 * tc + cl;
                const double ev = (x <= i) ? M[(int64_t)(P0 + x) * ld + P0 + i] : 0.0;
                o = __builtin_amdgcn_mfma_f64_16x16x4f64(ev, acc[ta][r], o, 0, 0, 0);
              }
            out[tc] = o;
          }
        }
#pragma unroll
        for (int ta = 0; ta < 4; ++ta)
#pragma unroll
          for (int r = 0; r < 4; ++r) Y[(int64_t)(P0 + 16 * ta + g + 4 * r) * ld + c0 + cl] = out[ta][r];
      }
      BAR();  // the panel's rows of Y complete before the next panel reads them
    }
    for (int t = wv; t < NB * (NB + 1) / 2; t += NW) {
      LANE_IDS();
      int I, J;
      tri_ij(t, I, J);
      d4 acc[4][4];
      zero_blk(acc);
      for (int P = I; P < NB; ++P) {
        if (I == J)
          gram_blkT<true, false>(acc, Y + (int64_t)64 * P * ld, ld, 64 * I, 64 * J, nullptr);
        else
          gram_blkT<false, false>(acc, Y + (int64_t)64 * P * ld, ld, 64 * I, 64 * J, nullptr);
      }
#pragma unroll
      for (int a_ = 0; a_ < 4; ++a_)
#pragma unroll
        for (int b_ = 0; b_ < 4; ++b_)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (I == J && b_ < a_) continue;
            const int i = 64 * I + 16 * b_ + cl, j = 64 * J + 16 * a_ + g + 4 * r;
            if (i < j) continue;  // upper half of a diagonal tile: its mirror is written
            const double v = acc[a_][b_][r];
            M[(int64_t)j * ld + i] = v;
            if (i != j) M[(int64_t)i * ld + j] = v;
          }
    }
    BAR();
  }

  // Blocked symmetric Gauss-Jordan sweep of the 64nb x 64nb symmetric matrix
  // whose lower triangle is stored in M (column-major, ld); leaves -M^-1 in the
  // lower triangle.  Panel P: thread (wave w, lane l) holds panel rows
  // 64P + w + 8q (q < 8) at columns 64t + l; at step c the owner of row c
  // publishes it through LDS (the pivot column is the same row by symmetry,
  // which the update keeps exact: one product per (i,j)/(j,i) pair) and records
  // it in Yp.  Pivot d = the Schur complement = (Cholesky diagonal)^2, so the
  // failure test is the one LAPACK potrf applies (d <= 0 or NaN).  The other
  // blocks get M_IJ -= sum_c rc_c[I]' rc_c[J] / d_c once per panel (MFMA).
  template <int nb>
  __device__ bool sweep_nb(gdbl* M, int ld) {
    // members copied to locals: the step loop has a barrier in it, after which
    // members (this is a stack object once sweep is an out-of-line call) would
    // be reloaded from scratch
    const int rr = wv, ln = lane, t0 = tid, o_row = L.o_row, RW = L.RW;
    for (int P = 0; P < nb; ++P) {
      const int P0 = 64 * P;
      gdbl* const Y = Yp + (int64_t)P * 64 * RW;  // this panel's pivot rows
      gdbl* const rv = Rv + P0;                    // and -1/d of its pivots
      // Catch-up of row block P: its blocks receive the Gram updates of the
      // earlier panels they have not seen (block (t, P), t >= P: panels [0, P);
      // block (P, t), t < P: panels (t, P) -- panel t swept it as part of row t)
      for (int t = rr; t < nb; t += NW) {
        const int I = t > P ? t : P, J = t > P ? P : t;
        const int qlo = t < P ? t + 1 : 0;
        if (qlo >= P) continue;
        d4 acc[4][4];
        if (I == J) {
          load_blkT<true>(acc, M, ld, 64 * I, 64 * J);
          for (int Q = qlo; Q < P; ++Q)
            gram_blkT<true>(acc, Yp + (int64_t)Q * 64 * RW, RW, 64 * I, 64 * J, Rv + 64 * Q);
          store_blkT<true>(acc, M, ld, 64 * I, 64 * J);
        } else {
          load_blkT(acc, M, ld, 64 * I, 64 * J);
          for (int Q = qlo; Q < P; ++Q)
            gram_blkT(acc, Yp + (int64_t)Q * 64 * RW, RW, 64 * I, 64 * J, Rv + 64 * Q);
          store_blkT(acc, M, ld, 64 * I, 64 * J);
        }
      }
      BAR();
      LSTAMP(NSTAMP + 1 + 0);
#if SOCP_LG_PANEL
      const bool ok = panel_tiles<nb>(M, ld, P);
      LSTAMP(NSTAMP + 1 + 1);
      if (!ok) return false;
#else
      double Z[8][nb];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int x = P0 + rr + 8 * q;
#pragma unroll
        for (int t = 0; t < nb; ++t) {
          const int y = 64 * t + ln;  // element (x, y) from the lower triangle
          Z[q][t] = M[(y <= x) ? (int64_t)y * ld + x : (int64_t)x * ld + y];
        }
      }
      bool ok = true;
      for (int c = 0; c < 64; ++c) {
        const int buf = o_row + (c & 1) * RW;
        if (rr == (c & 7)) {
          const int qc = c >> 3;
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            if (q == qc) {
#pragma unroll
              for (int t = 0; t < nb; ++t) {
                LV(buf + 64 * t + ln) = Z[q][t];
                Y[(int64_t)c * RW + 64 * t + ln] = Z[q][t];  // coalesced row store
              }
            }
          }
        }
        LDS_BAR();  // the pivot row's Yp / rv stores drain by the panel's BAR()
        const double d = LV(buf + P0 + c);
        ok = ok && (d > 0.0);
        const double r = 1.0 / d;
        if (t0 == 0) rv[c] = -r;
        double rowv[nb], colv[8];
#pragma unroll
        for (int t = 0; t < nb; ++t) rowv[t] = LV(buf + 64 * t + ln);
#pragma unroll
        for (int q = 0; q < 8; ++q) colv[q] = LV(buf + P0 + rr + 8 * q);
        // rank-1 update of every element as (col_i sqrt(r)) (row_j sqrt(r)): one
        // FMA per element, and (i,j), (j,i) multiply the same two numbers, so the
        // diagonal block stays exactly symmetric (r = 1/d > 0 whenever ok holds);
        // then the pivot column (block P, lane c: a select) and the pivot row
        // (one register row of one wavefront)
        const double sr = sqrt(r);
        double rsq[nb], csq[8];
#pragma unroll
        for (int t = 0; t < nb; ++t) rsq[t] = rowv[t] * sr;
#pragma unroll
        for (int q = 0; q < 8; ++q) csq[q] = colv[q] * sr;
#pragma unroll
        for (int q = 0; q < 8; ++q)
#pragma unroll
          for (int t = 0; t < nb; ++t) Z[q][t] = fma(-csq[q], rsq[t], Z[q][t]);
        const bool lc = ln == c;
#pragma unroll
        for (int t = 0; t < nb; ++t)
          if (t == P) {
#pragma unroll
            for (int q = 0; q < 8; ++q) Z[q][t] = lc ? colv[q] * r : Z[q][t];
          }
        if (rr == (c & 7)) {
          const int qc = c >> 3;
#pragma unroll
          for (int q = 0; q < 8; ++q)
            if (q == qc) {
#pragma unroll
              for (int t = 0; t < nb; ++t) Z[q][t] = (t == P && lc) ? -r : rowv[t] * r;
            }
        }
      }
      BAR();  // Yp and the pivot reciprocals complete
      LSTAMP(NSTAMP + 1 + 1);
      if (!ok) return false;
      {
        // addresses recomputed from a fresh lane id: reusing the load's would
        // keep 64 of them live (spilled) across the step loop
        const int lf = lane_fresh();
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int x = P0 + rr + 8 * q;
#pragma unroll
          for (int t = 0; t < nb; ++t) {
            const int y = 64 * t + lf;
            M[(y <= x) ? (int64_t)y * ld + x : (int64_t)x * ld + y] = Z[q][t];
          }
        }
      }
#endif
      BAR();  // panel P written back before the next catch-up reads its neighbours
      LSTAMP(NSTAMP + 1 + 2);
    }
    // Final catch-up: block (I, J), I >= J, has seen the panels up to I; it
    // receives those after I.  Each block is thus read and written 3 times per
    // sweep instead of once per panel; the Gram products (and their order) are
    // the right-looking sweep's, so the result is the same to the bit.
    const int ng = nb * (nb + 1) / 2;
    for (int t = rr; t < ng; t += NW) {
      int I, J;
      tri_ij(t, I, J);
      if (I + 1 >= nb) continue;
      d4 acc[4][4];
      if (I == J) {
        load_blkT<true>(acc, M, ld, 64 * I, 64 * J);
        for (int Q = I + 1; Q < nb; ++Q)
          gram_blkT<true>(acc, Yp + (int64_t)Q * 64 * RW, RW, 64 * I, 64 * J, Rv + 64 * Q);
        store_blkT<true>(acc, M, ld, 64 * I, 64 * J);
      } else {
        load_blkT(acc, M, ld, 64 * I, 64 * J);
        for (int Q = I + 1; Q < nb; ++Q)
          gram_blkT(acc, Yp + (int64_t)Q * 64 * RW, RW, 64 * I, 64 * J, Rv + 64 * Q);
        store_blkT(acc, M, ld, 64 * I, 64 * J);
      }
    }
    BAR();
    LSTAMP(NSTAMP + 1 + 3);
    return true;
  }

  // nb (= ld / 64) as a template constant: the panel row is then a fixed
  // register array with no per-element predicates
  __device__ bool sweep(gdbl* M, int ld) {
    switch (ld / 64) {
      case 1: return sweep_nb<1>(M, ld);
      case 2: return sweep_nb<2>(M, ld);
      case 3: return sweep_nb<3>(M, ld);
      case 4: return sweep_nb<4>(M, ld);
      case 5: return sweep_nb<5>(M, ld);
      case 6: return sweep_nb<6>(M, ld);
      case 7: return sweep_nb<7>(M, ld);
      default: return sweep_nb<8>(M, ld);
    }
  }

  // M (lower triangle = -X^-1) -> X^-1 in both triangles
  // by 64x64 lower blocks in the transposed MFMA orientation: the block is
  // read and rewritten in 128-byte rows, its mirror written in 32-byte runs
  // (element-wise mirroring wrote 8 bytes per cache line)
  __device__ void finalize_sym(gdbl* M, int ld) {
    const int NB = ld / 64, g = lane >> 4, cl = lane & 15;
    for (int t = wv; t < NB * (NB + 1) / 2; t += NW) {
      int I, J;
      tri_ij(t, I, J);
      d4 acc[4][4];
      if (I == J)
        load_blkT<true>(acc, M, ld, 64 * I, 64 * J);
      else
        load_blkT(acc, M, ld, 64 * I, 64 * J);
#pragma unroll
      for (int a_ = 0; a_ < 4; ++a_)
#pragma unroll
        for (int b_ = 0; b_ < 4; ++b_)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            if (I == J && b_ < a_) continue;
            const int i = 64 * I + 16 * b_ + cl, j = 64 * J + 16 * a_ + g + 4 * r;
            if (i < j) continue;  // upper half of a diagonal tile: not maintained
            const double v = -acc[a_][b_][r];
            M[(int64_t)j * ld + i] = v;
            if (i != j) M[(int64_t)i * ld + j] = v;
          }
    }
    BAR();
  }

  // setup_iter (densesolver.jl:41-52): H (+A'A), Li = H^-1, T = Li A', S = A T, S^-1
  __device__ int factor(bool addAA, bool h_only) {
    LSTAMP(SP_OTHER);
    const bool stg = form_X_fast_ok() && staged_ok();
    for (int rep = 0; rep < LREP(1); ++rep)
      if (!form_X_fast(stg)) form_X();
    LSTAMP(SP_U);
    for (int rep = 0; rep < LREP(2); ++rep) {
      if (stg)
        form_H_staged(addAA);
      else
        form_H(addAA);
    }
    LSTAMP(SP_SYRK);
    if constexpr (CHOL) {
    if (!chol(Hm, L.NPAD)) return ST_CHOL_H;
    if (h_only) return 0;
    LSTAMP(SP_SWEEP_H);
    for (int rep = 0; rep < LREP(32); ++rep) {
      chol_fwd_multi(Hm, L.NPAD);
      form_S_gram();
    }
    LSTAMP(SP_SCHUR);
    } else {
    if constexpr (INV_CHOL) {
      if (!chol(Hm, L.NPAD)) return ST_CHOL_H;
      if (h_only) return 0;
      chol_inverse(Hm, L.NPAD);
    } else {
      if (!sweep(Hm, L.NPAD)) return ST_CHOL_H;
      if (h_only) return 0;
      finalize_sym(Hm, L.NPAD);
    }
    LSTAMP(NSTAMP + 1 + 4);
    LSTAMP(SP_SWEEP_H);
    const int NB = L.NPAD / 64, MB = L.MPAD / 64;
    for (int t = wv; t < NB * MB; t += NW) {
      const int I = t / MB, J = t - I * MB;
      d4 acc[4][4];
      zero_blk(acc);
      blk_gemm(acc, Hm, At, L.NPAD, 64 * I, 64 * J, L.NPAD, false, -1);
      store_blk(acc, Tm, L.NPAD, 64 * I, 64 * J, NOPAD);
    }
    BAR();
    for (int t = wv; t < MB * (MB + 1) / 2; t += NW) {
      int I, J;
      tri_ij(t, I, J);
      d4 acc[4][4];
      zero_blk(acc);
      blk_gemm(acc, At, Tm, L.NPAD, 64 * I, 64 * J, L.NPAD, false, -1);
      store_blk(acc, Sm, L.MPAD, 64 * I, 64 * J, m);
    }
    BAR();
    LSTAMP(SP_SCHUR);
    }
    if (CHOL && L.MPAD > 64 * LARGE_NB_MAX) {
      // m > 512: S = L_S L_S' in place (the windowed panels of chol_wide); the
      // solves apply S^-1 as two triangular solves.  cholesky! of S fails
      // where this does (densesolver.jl:51)
      if (!chol(Sm, L.MPAD)) return ST_CHOL_S;
      LSTAMP(SP_SCHUR);
      return 0;
    }
    if constexpr (INV_CHOL) {
      if (!chol(Sm, L.MPAD)) return ST_CHOL_S;
      chol_inverse(Sm, L.MPAD);
    } else {
      if (!sweep(Sm, L.MPAD)) return ST_CHOL_S;
      finalize_sym(Sm, L.MPAD);
    }
    LSTAMP(SP_SCHUR);
    return 0;
  }

  // ------------------------------------------------------------ mat-vecs
  // out[j] = (G' vin)[j] (+ add[j]) for j < n: a wavefront takes CG columns
  // Fast path (k <= 64 GT_R): a wavefront loads its CG columns whole -- every
  // load of the pass in flight at once (GT_R x CG per lane) -- instead of one
  // 64-row step of the CG columns per memory round trip.
  static constexpr int GT_R = 10;
#ifndef SOCP_LG_GT_FAST
#define SOCP_LG_GT_FAST 1
#endif
  __device__ void gemv_Gt(int vin, int vout, int vadd) {
    LSTAMP(SP_SOLVE);
    if (SOCP_LG_GT_FAST && k <= 64 * GT_R) {
      double vr[GT_R];
#pragma unroll
      for (int r = 0; r < GT_R; ++r) vr[r] = (lane + 64 * r < k) ? LV(vin + lane + 64 * r) : 0.0;
      for (int j0 = CG * wv; j0 < n; j0 += CG * NW) {
        gcdbl* g0 = Gp + (int64_t)j0 * k;
        const int nl = n - j0;
        double gv[CG][GT_R];
#pragma unroll
        for (int u = 0; u < CG; ++u)
#pragma unroll
          for (int r = 0; r < GT_R; ++r) {
            const int row = lane + 64 * r;
            gv[u][r] = (row < k) ? g0[(int64_t)(u < nl ? u : 0) * k + row] : 0.0;
          }
        double acc[CG];
#pragma unroll
        for (int u = 0; u < CG; ++u) {
          acc[u] = 0.0;
#pragma unroll
          for (int r = 0; r < GT_R; ++r) acc[u] = fma(gv[u][r], vr[r], acc[u]);
        }
#pragma unroll
        for (int u = 0; u < CG; ++u) {
          const double s = wave_sum(acc[u]);
          if (lane == 0 && j0 + u < n) LV(vout + j0 + u) = (vadd >= 0) ? s + LV(vadd + j0 + u) : s;
        }
      }
      BAR();
      LSTAMP(NSTAMP + 1 + 5);
      return;
    }
    for (int j0 = CG * wv; j0 < n; j0 += CG * NW) {
      gcdbl* g0 = Gp + (int64_t)j0 * k;
      const int nl = n - j0;  // live columns u < nl (dead ones re-read column j0)
      double acc[CG];
#pragma unroll
      for (int u = 0; u < CG; ++u) acc[u] = 0.0;
      for (int i = lane; i < k; i += 64) {
        const double v = LV(vin + i);
#pragma unroll
        for (int u = 0; u < CG; ++u) acc[u] = fma(g0[(int64_t)(u < nl ? u : 0) * k + i], v, acc[u]);
      }
#pragma unroll
      for (int u = 0; u < CG; ++u) {
        const double s = wave_sum(acc[u]);
        if (lane == 0 && j0 + u < n) LV(vout + j0 + u) = (vadd >= 0) ? s + LV(vadd + j0 + u) : s;
      }
    }
    BAR();
    LSTAMP(NSTAMP + 1 + 5);
  }
  // The residuals' two G products in one pass over G (solver.jl:110-118):
  // vout = G'zin and gout[i] = (G xin)[i] + add[i] - sub[i].  As gemv_Gt's fast
  // path, a wavefront holds CGM columns whole; it also accumulates its lanes'
  // rows' share of G xin over its columns, and the eight per-wave partial
  // vectors meet in the LDS region that is dead outside a solve (the seven
  // dead k-vectors and the sweep scratch, from 0), summed in wave order.
  // Returns false (the two separate passes run instead) where the shape
  // does not fit that.
  static constexpr int CGM = 4;
  __device__ bool gemv_GtG(int zin, int vout, int xin, int add, int sub, int gout) {
    const int KP = L.KP;
    if (!SOCP_LG_GT_FAST || k > 64 * GT_R || L.o_kvd != 0 || 8 * KP > L.o_part + 8 * L.MPAD) return false;
    LSTAMP(SP_SOLVE);
    double vr[GT_R], pr[GT_R];
#pragma unroll
    for (int r = 0; r < GT_R; ++r) {
      vr[r] = (lane + 64 * r < k) ? LV(zin + lane + 64 * r) : 0.0;
      pr[r] = 0.0;
    }
    for (int j0 = CGM * wv; j0 < n; j0 += CGM * NW) {
      gcdbl* g0 = Gp + (int64_t)j0 * k;
      const int nl = n - j0;
      double gv[CGM][GT_R], xs[CGM];
#pragma unroll
      for (int u = 0; u < CGM; ++u) {
        xs[u] = u < nl ? LV(xin + j0 + u) : 0.0;
#pragma unroll
        for (int r = 0; r < GT_R; ++r) {
          const int row = lane + 64 * r;
          gv[u][r] = (row < k) ? g0[(int64_t)(u < nl ? u : 0) * k + row] : 0.0;
        }
      }
      double acc[CGM];
#pragma unroll
      for (int u = 0; u < CGM; ++u) {
        acc[u] = 0.0;
#pragma unroll
        for (int r = 0; r < GT_R; ++r) acc[u] = fma(gv[u][r], vr[r], acc[u]);
      }
#pragma unroll
      for (int r = 0; r < GT_R; ++r)
#pragma unroll
        for (int u = 0; u < CGM; ++u) pr[r] = fma(gv[u][r], xs[u], pr[r]);
#pragma unroll
      for (int u = 0; u < CGM; ++u) {
        const double sm = wave_sum(acc[u]);
        if (lane == 0 && j0 + u < n) LV(vout + j0 + u) = sm;
      }
    }
    const int part = L.o_kvd;
#pragma unroll
    for (int r = 0; r < GT_R; ++r)
      if (lane + 64 * r < KP) LV(part + wv * KP + lane + 64 * r) = pr[r];
    BAR();
    for (int i = tid; i < k; i += NTH) {
      double sm = 0.0;
#pragma unroll
      for (int w = 0; w < NW; ++w) sm += LV(part + w * KP + i);
      if (add >= 0) sm = sm + LV(add + i);
      LV(gout + i) = sm - LV(sub + i);
    }
    BAR();
    for (int e = tid; e < 7 * KP; e += NTH) LV(part + e) = 0.0;  // the dead k-vectors read 0 again
    BAR();
    LSTAMP(NSTAMP + 1 + 5);
    return true;
  }
  // out[i] = (G u)[i] (+ add[i]) - sub[i] for i < k: one thread per row.  When
  // NTH < k <= 2 NTH the rows past the first NTH are split over T = NTH/(k-NTH)
  // threads of one wavefront each (column slices, a shuffle sum), so the second
  // round costs 1/T of the first instead of a whole one with most threads idle.
  __device__ void gemv_G(int u, int add, int sub, int out) {
    LSTAMP(SP_SOLVE);
    const int r2 = k - NTH;
    int T = 0;
    if (r2 > 0 && r2 <= NTH) {
      T = 1;
      while (T < 64 && T * 2 * r2 <= NTH) T *= 2;
    }
    const int i1 = T > 1 ? (k < NTH ? k : NTH) : k;  // rows done one thread each
    for (int i = tid; i < i1; i += NTH) {
      double acc = 0.0;
#pragma unroll 16
      for (int j = 0; j < n; ++j) acc = fma(Gp[(int64_t)j * k + i], LV(u + j), acc);
      if (add >= 0) acc = acc + LV(add + i);
      LV(out + i) = acc - LV(sub + i);
    }
    if (T > 1) {
      const int i = NTH + tid / T, q = tid % T;  // T | 64: a row's threads share a wavefront
      const int js = (n + T - 1) / T, j0 = q * js, j1 = j0 + js < n ? j0 + js : n;
      const bool live = i < k;
      double acc = 0.0;
      if (live) {
#pragma unroll 8
        for (int j = j0; j < j1; ++j) acc = fma(Gp[(int64_t)j * k + i], LV(u + j), acc);
      }
      for (int d = 1; d < T; d *= 2) acc += __shfl_xor(acc, d, 64);
      if (live && q == 0) {
        if (add >= 0) acc = acc + LV(add + i);
        LV(out + i) = acc - LV(sub + i);
      }
    }
    BAR();
    LSTAMP(NSTAMP + 1 + 7);
  }
  // (A' v)[j] for one j (thread per column; At rows are contiguous in j)
  __device__ __forceinline__ double At_dot(int v, int j) const {
    double acc = 0.0;
    for (int r = 0; r < m; ++r) acc = fma(At[(int64_t)r * L.NPAD + j], LV(v + r), acc);
    return acc;
  }
  // out[r] = (A u)[r] - sub[r] for r < m; returns this thread's share of |out|^2.
  // Mt: A' row-major (Ap), or Z = L^-1 A' (Tm, the Cholesky path): out = Z'u - sub.
  __device__ double A_mv(int u, int sub, int out) { return mat_mv(Ap, u, sub, out); }
  __device__ double mat_mv(gcdbl* Mt, int u, int sub, int out) {
    for (int r = lane; r < L.MPAD; r += 64) {
      double acc = 0.0;
      for (int j = wv; j < n; j += NW) acc = fma(Mt[(int64_t)j * L.MPAD + r], LV(u + j), acc);
      LV(L.o_part + wv * L.MPAD + r) = acc;
    }
    BAR();
    double sq = 0.0;
    for (int r = tid; r < m; r += NTH) {
      double s = 0.0;
#pragma unroll
      for (int w = 0; w < NW; ++w) s += LV(L.o_part + w * L.MPAD + r);
      const double v = s - LV(sub + r);
      LV(out + r) = v;
      sq = fma(v, v, sq);
    }
    BAR();
    return sq;
  }
  // out = M vin for a full symmetric column-major M (thread per row)
  __device__ void symv(gcdbl* M, int ld, int vin, int vout) {
    LSTAMP(SP_SOLVE);
    for (int i = tid; i < ld; i += NTH) {
      double acc = 0.0;
#pragma unroll 16
      for (int j = 0; j < ld; ++j) acc = fma(M[(int64_t)j * ld + i], LV(vin + j), acc);
      LV(vout + i) = acc;
    }
    BAR();
    LSTAMP(NSTAMP + 1 + 6);
  }

  // Triangular solves against the in-place factor of chol_nb (L below the
  // diagonal blocks, E_P = L_PP^-1 in them), 64 rows per step.  Rows >= n
  // (padding) are never read.
  // out = L^-1 in: r = in_P - L_P,<P out_<P (lanes = rows, wavefronts split
  // the columns; partial sums through LDS), out_P = E_P r.
  // (dim: the factor's order -- n for H, m for S; ld = its padded order)
  __device__ void trsv_fwd(gcdbl* Lm, int ld, int vin, int vout, int dim) {
    const int NB = ld / 64, p1 = L.o_part, p2 = L.o_fx, n = dim;
    LSTAMP(SP_SOLVE);
    for (int P = 0; P < NB; ++P) {
      const int P0 = 64 * P, i = P0 + lane;
      double acc = 0.0;
      if (i < n) {
#pragma unroll 8
        for (int y = wv; y < P0; y += NW) acc = fma(Lm[(int64_t)y * ld + i], LV(vout + y), acc);
      }
      LV(p1 + wv * 64 + lane) = acc;
      LDS_BAR();
      acc = 0.0;
      {
        // the panel's 64 / NW columns of this wavefront: their loads first
        // (one memory round trip), then the same FMA chain as before
        constexpr int XW = 64 / NW;
        double lx[XW];
#pragma unroll
        for (int j = 0; j < XW; ++j) {
          const int x = wv + NW * j;
          lx[j] = (P0 + x < n && x <= lane && i < n) ? Lm[(int64_t)(P0 + x) * ld + i] : 0.0;
        }
#pragma unroll
        for (int j = 0; j < XW; ++j) {
          const int x = wv + NW * j;
          if (P0 + x >= n) break;  // wave-uniform
          double r = LV(vin + P0 + x);
#pragma unroll
          for (int w = 0; w < NW; ++w) r -= LV(p1 + w * 64 + x);
          if (x <= lane && i < n) acc = fma(lx[j], r, acc);
        }
      }
      LV(p2 + wv * 64 + lane) = acc;
      LDS_BAR();
      if (wv == 0 && i < n) {
        double u = 0.0;
#pragma unroll
        for (int w = 0; w < NW; ++w) u += LV(p2 + w * 64 + lane);
        LV(vout + i) = u;
      }
      LDS_BAR();
    }
    LSTAMP(NSTAMP + 1 + 6);
  }
  // out = L^-T in, last block first: r = in_P - L_>P,P' out_>P, out_P = E_P' r.
  // Both products read columns of L / E (contiguous): 16 lanes per column,
  // four columns per wavefront step.
  __device__ void trsv_bwd(gcdbl* Lm, int ld, int vin, int vout, int dim) {
    const int NB = ld / 64, p1 = L.o_part, q = lane >> 4, c = lane & 15, n = dim;
    LSTAMP(SP_SOLVE);
    for (int P = NB - 1; P >= 0; --P) {
      const int P0 = 64 * P;
      for (int i = 4 * wv + q; i < 64; i += 4 * NW) {
        double acc = 0.0;
#pragma unroll 4
        for (int x = P0 + 64 + c; x < n; x += 16) acc = fma(Lm[(int64_t)(P0 + i) * ld + x], LV(vout + x), acc);
        acc = row16_sum(acc);
        if (c == 0) LV(p1 + i) = (P0 + i < n) ? LV(vin + P0 + i) - acc : 0.0;
      }
      LDS_BAR();
      for (int i = 4 * wv + q; i < 64; i += 4 * NW) {
        double acc = 0.0;
#pragma unroll
        for (int s_ = 0; s_ < 4; ++s_) {
          const int x = c + 16 * s_;
          if (x >= i && P0 + x < n) acc = fma(Lm[(int64_t)(P0 + i) * ld + P0 + x], LV(p1 + x), acc);
        }
        acc = row16_sum(acc);
        if (c == 0 && P0 + i < n) LV(vout + P0 + i) = acc;
      }
      LDS_BAR();
    }
    LSTAMP(NSTAMP + 1 + 6);
  }
  // out[j] = u[j] + (Z m)[j], j < n (Z row-major in Tm: 16 lanes per row)
  __device__ void z_mv_add(int u, int mv, int out) {
    const int q = lane >> 4, c = lane & 15;
    for (int j0 = 4 * wv; j0 < n; j0 += 4 * NW) {
      const int j = j0 + q;
      double acc = 0.0;
      if (j < n)
        for (int r = c; r < m; r += 16) acc = fma(Tm[(int64_t)j * L.MPAD + r], LV(mv + r), acc);
      acc = row16_sum(acc);
      if (c == 0 && j < n) LV(out + j) = LV(u + j) + acc;
    }
    LDS_BAR();
  }

  // rd = A'y + G'z + c, rp = Ax - b, rz = Gx + s - h (solver.jl:109-118)
  __device__ void residuals(double& nd, double& np_, double& gap) {
    bool merged = false;
    for (int rep = 0; rep < LREP(64); ++rep) merged = gemv_GtG(Z_, TN, X_, S_, H_, DZ);  // G'z and Gx + s - h in one G pass
    if (!merged) gemv_Gt(Z_, TN, -1);
    double d2 = 0.0;
    for (int j = tid; j < n; j += NTH) {
      const double v = (At_dot(Y_, j) + LV(TN + j)) + LV(C_ + j);
      LV(RD + j) = v;
      d2 = fma(v, v, d2);
    }
    const double p2 = A_mv(X_, B_, RP);
    if (!merged) gemv_G(X_, S_, H_, DZ);
    double zs = 0.0;
    for (int i = tid; i < k; i += NTH) zs += LV(Z_ + i) * LV(S_ + i);
    nd = sqrt(block_sum(d2));
    np_ = sqrt(block_sum(p2));
    gap = block_sum(zs);
  }

  // The matrix part of solve_kkt (densesolver.jl:66-85): n0 = GWiWi*k2 + dx
  // (+A'dy if sing); m0 = A Li n0 - dy; cy = S^-1 m0; m0 = sing ? dy - cy : -cy
  // (init: -cy); cx = Li (n0 + A'm0), taken as Li n0 + (Li A') m0; k1 = G cx - k2.
  // In: RD RP T2 K2.  Out: RX RY K1.
  __device__ void solve_matrix_part(bool init) {
    for (int rep = 0; rep < LREP(4); ++rep) gemv_Gt(T2, N0, RD);
    if (sing) {
      for (int j = tid; j < n; j += NTH) LV(N0 + j) = LV(N0 + j) + At_dot(RP, j);
      BAR();
    }
    if constexpr (CHOL) {
    // Li = L^-T L^-1: u = L^-1 n0; m0 = A Li n0 - dy = Z'u - dy; cy = S^-1 m0;
    // cx = Li (n0 + A'm0) = L^-T (u + Z m0)
    for (int rep = 0; rep < LREP(16); ++rep) trsv_fwd(Hm, L.NPAD, N0, TN, n);
    mat_mv(Tm, TN, RP, M0);
    if (L.MPAD > 64 * LARGE_NB_MAX) {  // S = L_S L_S' (factor() factors S beyond the sweep's reach)
      trsv_fwd(Sm, L.MPAD, M0, M0, m);
      trsv_bwd(Sm, L.MPAD, M0, RY, m);
    } else {
      symv(Sm, L.MPAD, M0, RY);
    }
    for (int r = tid; r < m; r += NTH) LV(M0 + r) = (sing && !init) ? LV(RP + r) - LV(RY + r) : -LV(RY + r);
    BAR();
    z_mv_add(TN, M0, N0);
    for (int rep = 0; rep < LREP(16); ++rep) trsv_bwd(Hm, L.NPAD, N0, RX, n);
    } else {
    symv(Hm, L.NPAD, N0, TN);
    A_mv(TN, RP, M0);
    symv(Sm, L.MPAD, M0, RY);
    for (int r = tid; r < m; r += NTH) LV(M0 + r) = (sing && !init) ? LV(RP + r) - LV(RY + r) : -LV(RY + r);
    BAR();
    // cx = Li (n0 + A'm0) = Li n0 + (Li A') m0: one pass over Li per solve
    // (T = Li A' is the factor's, column-major NPAD x MPAD)
    for (int j = tid; j < n; j += NTH) {
      double acc = 0.0;
      for (int r = 0; r < m; ++r) acc = fma(Tm[(int64_t)r * L.NPAD + j], LV(M0 + r), acc);
      LV(RX + j) = LV(TN + j) + acc;
    }
    BAR();
    }
    for (int rep = 0; rep < LREP(8); ++rep) gemv_G(RX, -1, K2, K1);
  }

  // ------------------------------------------------------------- driver
  // solve_socp (solver.jl:40-153) for problem p: the register kernel's control
  // flow and status rules.
  __device__ void run(int64_t p) {
    LSTAMP(SP_OTHER);
    if (rec0) set_record(p);
    load(p);
    LSTAMP(SP_LOAD);
    int status = ST_MAXIT, iters = 0;
    double nd = NAN, np_ = NAN, gap = NAN, ll = 0.0;
    bool dm_aa = false;
    if (a.mode == MODE_SOLVEKKT) {  // solve_kkt against the setup_iter record
      const int st0 = (int)Vr[3 * L.KP + 12 * MAXC + 1];
      if (st0) {  // setup_iter failed for this problem: NaN solution, its status
        for (int j = tid; j < n; j += NTH) a.cx[p * n + j] = NAN;
        for (int i = tid; i < m; i += NTH) a.cy[p * m + i] = NAN;
        for (int i = tid; i < k; i += NTH) {
          a.cz[p * k + i] = NAN;
          a.cs[p * k + i] = NAN;
        }
        if (tid == 0) a.status[p] = st0;
        BAR();
        return;
      }
      load_record();
      for (int i = tid; i < k; i += NTH) {
        LV(DZ + i) = a.dz[p * k + i];
        LV(DS + i) = a.ds[p * k + i];
      }
      for (int j = tid; j < n; j += NTH) LV(RD + j) = a.dx[p * n + j];
      for (int i = tid; i < m; i += NTH) LV(RP + i) = a.dy[p * m + i];
      BAR();
      solve_head();
      solve_matrix_part(false);
      int dom = 0;
      solve_tail(false, dm_aa, dom);
      for (int j = tid; j < n; j += NTH) a.cx[p * n + j] = LV(RX + j);
      for (int i = tid; i < m; i += NTH) a.cy[p * m + i] = LV(RY + i);
      for (int i = tid; i < k; i += NTH) {
        a.cz[p * k + i] = LV(RZ + i);
        a.cs[p * k + i] = LV(RS + i);
      }
      if (tid == 0) a.status[p] = 0;
      BAR();
      return;
    }
    if (a.sing) {
      sing = a.sing[p] != 0;
    } else {  // Problem's `sing` (Socp.jl:49-56): does cholesky(G'G) fail?
      scaling_identity();
      sing = factor(false, true) == ST_CHOL_H;
    }
    if (a.mode == MODE_KKT || a.mode == MODE_SETUP) {
      for (int i = tid; i < k; i += NTH) {
        LV(S_ + i) = a.s[p * k + i];
        LV(Z_ + i) = a.z[p * k + i];
        if (a.mode == MODE_KKT) {
          LV(DZ + i) = a.dz[p * k + i];
          LV(DS + i) = a.ds[p * k + i];
        }
      }
      if (a.mode == MODE_KKT) {
        for (int j = tid; j < n; j += NTH) LV(RD + j) = a.dx[p * n + j];
        for (int i = tid; i < m; i += NTH) LV(RP + i) = a.dy[p * m + i];
      }
      BAR();
      if (scaling_op(ll, dm_aa, false)) {
        status = ST_DOMAIN;
      } else {
        const int f = factor(sing, false);
        if (f) {
          status = f;
        } else if (a.mode == MODE_SETUP) {
          store_record();
          status = 0;
        } else {
          solve_head();
          solve_matrix_part(false);
          int dom = 0;
          solve_tail(false, dm_aa, dom);
          status = 0;
          for (int j = tid; j < n; j += NTH) a.cx[p * n + j] = LV(RX + j);
          for (int i = tid; i < m; i += NTH) a.cy[p * m + i] = LV(RY + i);
          for (int i = tid; i < k; i += NTH) {
            a.cz[p * k + i] = LV(RZ + i);
            a.cs[p * k + i] = LV(RS + i);
          }
        }
      }
      if (tid == 0) {
        a.status[p] = status;
        if (a.mode == MODE_SETUP) Vr[3 * L.KP + 12 * MAXC + 1] = (double)status;
      }
      BAR();
      return;
    }
    bool go = true;
    if (a.flags & F_WARM) {
      for (int j = tid; j < n; j += NTH) LV(X_ + j) = a.x[p * n + j];
      for (int i = tid; i < m; i += NTH) LV(Y_ + i) = a.y[p * m + i];
      for (int i = tid; i < k; i += NTH) {
        LV(Z_ + i) = a.z[p * k + i];
        LV(S_ + i) = a.s[p * k + i];
      }
      BAR();
    } else {  // initial point: the KKT system with W = I (solver.jl:68-84), then the shift (:86-104)
      scaling_identity();
      for (int j = tid; j < n; j += NTH) LV(RD + j) = -LV(C_ + j);
      for (int i = tid; i < m; i += NTH) LV(RP + i) = LV(B_ + i);
      for (int i = tid; i < k; i += NTH) {
        LV(DZ + i) = LV(H_ + i);
        LV(DS + i) = 0.0;
      }
      BAR();
      const int f = factor(sing, false);
      if (f) {
        status = f;
        go = false;
      } else {
        solve_head();
        solve_matrix_part(true);
        int dom = 0;
        solve_tail(false, false, dom);
        double alphp, alphd;
        maxstep_op(RZ, alphp, alphd);
        for (int j = tid; j < n; j += NTH) LV(X_ + j) = LV(RX + j);
        for (int i = tid; i < m; i += NTH) LV(Y_ + i) = LV(RY + i);
        for (int i = tid; i < k; i += NTH) {
          const double iz = LV(RZ + i), e = e_of(i);
          LV(S_ + i) = (fabs(alphp) < a.init_eps) ? -iz : -iz + (1.0 + alphp) * e;
          LV(Z_ + i) = (fabs(alphd) < a.init_eps) ? iz : iz + (1.0 + alphd) * e;
        }
        BAR();
      }
    }
    int it = 0;
    while (go) {
      LSTAMP(SP_OTHER);
      if (it >= a.maxit && !a.res) break;  // no residuals after the last iteration (solver.jl:105-151)
      residuals(nd, np_, gap);
      LSTAMP(SP_RESID);
      if (it >= a.maxit) break;
      bool dm_it = false;
      for (int rep = 0; rep < LREP(128); ++rep) dm_it = scaling_op(ll, dm_aa, true);
      LSTAMP(SP_SCALING);
      if (dm_it) {
        status = ST_DOMAIN;
        break;
      }
      if (nd + np_ + gap < a.tol) {
        status = ST_CONVERGED;
        break;
      }
      for (int j = tid; j < n; j += NTH) LV(RD + j) = -LV(RD + j);
      for (int i = tid; i < m; i += NTH) LV(RP + i) = -LV(RP + i);
      for (int i = tid; i < k; i += NTH) {
        LV(DZ + i) = -LV(DZ + i);
        LV(DS + i) = -LV(DS + i);
      }
      BAR();
      const int f = factor(sing, false);
      if (f) {
        status = f;
        break;
      }
      LSTAMP(SP_OTHER);
      for (int rep = 0; rep < LREP(256); ++rep) solve_head();  // affine direction (solver.jl:125-130)
      LSTAMP(SP_VOP);
      solve_matrix_part(false);
      LSTAMP(SP_SOLVE);
      int dom = 0;
      double t = solve_tail(true, dm_aa, dom);
      LSTAMP(SP_VOP);
      if (dom) {
        status = ST_DOMAIN;
        break;
      }
      affine_post(t, ll);
      LSTAMP(SP_STEP);
      for (int rep = 0; rep < LREP(256); ++rep) solve_head();  // combined direction (solver.jl:141-145)
      LSTAMP(SP_VOP);
      solve_matrix_part(false);
      LSTAMP(SP_SOLVE);
      t = solve_tail(true, dm_aa, dom);
      LSTAMP(SP_VOP);
      if (dom) {
        status = ST_DOMAIN;
        break;
      }
      const double stp = t * a.step;  // step and update (solver.jl:146-150)
      for (int j = tid; j < n; j += NTH) LV(X_ + j) = LV(X_ + j) + LV(RX + j) * stp;
      for (int i = tid; i < m; i += NTH) LV(Y_ + i) = LV(Y_ + i) + LV(RY + i) * stp;
      for (int i = tid; i < k; i += NTH) {
        LV(Z_ + i) = LV(Z_ + i) + LV(RZ + i) * stp;
        LV(S_ + i) = LV(S_ + i) + LV(RS + i) * stp;
      }
      BAR();
      LSTAMP(SP_STEP);
      iters = ++it;
    }
    for (int j = tid; j < n; j += NTH) a.x[p * n + j] = LV(X_ + j);
    for (int i = tid; i < m; i += NTH) a.y[p * m + i] = LV(Y_ + i);
    for (int i = tid; i < k; i += NTH) {
      a.z[p * k + i] = LV(Z_ + i);
      a.s[p * k + i] = LV(S_ + i);
    }
    if (tid == 0) {
      if (a.res) {
        a.res[3 * p + 0] = nd;
        a.res[3 * p + 1] = np_;
        a.res[3 * p + 2] = gap;
      }
      a.iters[p] = iters;
      a.status[p] = status;
    }
    BAR();
    LSTAMP(SP_STORE);
#ifdef SOCP_DIAG
    if (!GV && tid == 0) reinterpret_cast<unsigned long long*>(lg_lds + L.o_red + 16)[NSTAMP] += iters;
#endif
  }
};

template <bool XI, bool GV>
__global__ void __launch_bounds__(NTH, 1) socp_large_kernel(LargeArgs args) {
  // the next problem index lives in dynamic LDS (slot 63 of the block-reduction
  // area; GV: slot 0 of the kernel's small LDS): no static LDS, so lg_lds
  // starts at LDS address 0 and the staged SYRK's DMA buffers lie in the
  // first 64 KiB
  Large<XI, GV> S(args);
  S.init_tables();
  const int pslot = GV ? 0 : S.L.o_red + 63;
  while (true) {
    if (threadIdx.x == 0) lg_lds[pslot] = (double)atomicAdd(args.a.counter, 1);
    __syncthreads();
    const int64_t p = (int64_t)lg_lds[pslot];
    __syncthreads();  // everyone has read pidx before thread 0 overwrites it
    if (p >= args.a.B) break;
    S.run(p);
  }
  S.flush_stamps();
}

#if SOCP_LG_GV_TU
// the global-vector kernels (socp_large_gv.o: this file with SOCP_LG_GV_TU=1)
template __global__ void socp_large_kernel<false, true>(LargeArgs);
template __global__ void socp_large_kernel<true, true>(LargeArgs);
}  // namespace lg
#else
extern template __global__ void socp_large_kernel<false, true>(LargeArgs);
extern template __global__ void socp_large_kernel<true, true>(LargeArgs);
}  // namespace lg

const void* large_kernel_ptr(bool xi, bool gv) {
  if (gv) return xi ? (const void*)&lg::socp_large_kernel<true, true> : (const void*)&lg::socp_large_kernel<false, true>;
  return xi ? (const void*)&lg::socp_large_kernel<true, false> : (const void*)&lg::socp_large_kernel<false, false>;
}
const char* large_kernel_name(bool xi, bool gv) {
  if (gv) return xi ? "socp_large_xi_gv_kernel" : "socp_large_gv_kernel";
  return xi ? "socp_large_xi_kernel" : "socp_large_kernel";
}
#endif

}  // namespace socp
