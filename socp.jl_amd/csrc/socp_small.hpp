// socp_small.hpp — the register-resident batched dense SOCP IPM kernel (gfx950).
//
// One 64-lane wavefront owns one problem for its whole solve (persistent
// one-wave blocks pull problem indices from an atomic work counter).  The
// problem's G (k x n, the dominant data: 48 KiB at n=64,k=96) is loaded from
// HBM once per solve and stays in AGPRs for every iteration, laid out as the
// B-operand fragment of v_mfma_f64_16x16x4_f64:
//     lane (g = lane>>4, cl = lane&15) holds G[4p+g][16q+cl] in G[p][q].
// Per iteration (reference solver.jl:105-151):
//   - NT scaling (scalings.jl:22-110) with per-cone segmented DPP scans;
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
// Code-size discipline: the driver is a micro-phase loop in which the cone
// vector op, the factorisation, the KKT solve body and the residuals each
// have exactly one inlined instance (no calls: a call would force the live
// H/Li tiles out of registers), keeping the instruction stream cache-resident.
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

// MODE_SETUP / MODE_SOLVEKKT: the two plugin calls of densesolver.jl
// (setup_iter :41-52 keeps scaling + H^-1 + S^-1 in a per-problem device
// record; solve_kkt :54-90 solves one right-hand side against it)
enum { MODE_SOLVE = 0, MODE_KKT = 1, MODE_SETUP = 2, MODE_SOLVEKKT = 3 };
enum { ST_CONVERGED = 0, ST_MAXIT = 1, ST_CHOL_H = 2, ST_CHOL_S = 3, ST_DOMAIN = 4 };
enum { F_WARM = 2 };

struct SmallArgs {
  int64_t B;
  int32_t n, m, k, nc;
  int32_t maxit, sigma_exp;
  double tol, step, init_eps;
  int32_t flags, mode, deg;
  int32_t al_rows;  // 1, 2 or 4 when every cone is 16, 32 or 64 long (so 16-lane-row aligned): register-only cone reductions; 0 otherwise
  const double *c, *A, *b, *G, *h;
  const uint8_t* sing;
  double *x, *y, *z, *s;
  int32_t *iters, *status;
  double* res;
  const double *dx, *dy, *dz, *ds;
  double *cx, *cy, *cz, *cs;
  int32_t* counter;
  double* dbg;                 // optional (KKT mode): per problem H[n*n], Li[n*n], lam[k], wb[k]
  unsigned long long* stamps;  // SOCP_DIAG builds: per-phase cycle totals
  ConeTable cones;
  double* rec;                 // MODE_SETUP / MODE_SOLVEKKT: per-problem factor records
  int64_t rec_stride;          // doubles per record
};

// ------------------------------------------------------------ LDS layout
// Fixed region (independent of the template shape):
#ifdef SOCP_DIAG
#define SOCP_NSTAMP_SLOTS 24
#else
#define SOCP_NSTAMP_SLOTS 0
#endif
enum : int {
  O_COFF = 0,                // cone offs[NCS]
  O_CDIM = O_COFF + NCS,     // cone dim[NCS]
  O_CKIND = O_CDIM + NCS,    // cone kind[NCS]
  O_CC = O_CKIND + NCS,        // per-cone constants of the current scaling [NCC][NCS]
  O_PART = O_CC + 20 * NCS,    // segment partials [NVMAX = 6][NCS][2 slots] (zero where unused)
  O_TOTC = O_PART + 6 * NCS * 2,  // per-cone results [4][NCS]
  O_STAMPS = O_TOTC + 4 * NCS,  // diagnostic build only: per-phase cycle totals of this wave [24]
  O_FIXED = O_STAMPS + SOCP_NSTAMP_SLOTS  // then (Shape): rcode[KP], 17 k-vectors KS apart, ...
};
constexpr int NKV = 17;
#ifndef SOCP_SYRK_UBT
#define SOCP_SYRK_UBT 1  // the SYRK's U-row addresses from a launch-wide table (0: from the codes)
#endif
// per-cone constants (SOC cones), recomputed by every scaling:
//   MU = mu, IMU = 1/mu, WB0 = wbar_0, I1 = 1/(1+wbar_0), W2 = |wbar_1|^2,
//   L0 = lambda_0, AA = lambda_0^2 - |lambda_1|^2 (iprod!'s `a`, vectors.jl:105),
//   IAA = 1/AA, IL0 = 1/lambda_0, IL0AA = 1/(lambda_0 AA),
//   SA = 1/sqrt(AA) (scmax's `a`, mats.jl:66), SAL = 1/(SA lambda_0 + 1),
//   WL = wbar_1'lambda_1; AS, AZ, BS, BZ: the tail rows of wbar and lambda as
//   wbar_i = AS s_i - AZ z_i, lambda_i = BS s_i + BZ z_i (scalings.jl:57-97);
// per solve: DLT = wbar_1'k0_1 of the current KKT solve's k0 (solve_head ->
// solve_tail), KK = the cone's kt2'kt3 (head of kt2 o kt3, solve_tail -> affine_post)
enum : int { CC_MU, CC_IMU, CC_WB0, CC_I1, CC_W2, CC_L0, CC_AA, CC_IAA, CC_IL0, CC_IL0AA, CC_SA,
             CC_SAL, CC_WL, CC_AS, CC_AZ, CC_BS, CC_BZ, CC_DLT, CC_KK };
__host__ __device__ constexpr int cc(int q, int c) { return O_CC + q * NCS + c; }
// k-vector ids (IL: 1/lambda_i of the POC elements).  KV_RZ .. KV_T2 are
// dead while a factorisation runs (the previous solve's results are consumed,
// the next solve's temporaries not yet written): the Cholesky shapes' tile
// transpose buffer lives there (Shape::O_TB).
enum : int { KV_H, KV_Z, KV_S, KV_DZ, KV_DS, KV_LAM, KV_WB, KV_CA, KV_CB, KV_IL, KV_RZ, KV_RS, KV_K0,
             KV_K1, KV_K2, KV_T1, KV_T2 };
constexpr int NKV_DEAD = KV_T2 - KV_RZ + 1;

// the A block's leading dimension (Shape::LDA)
__host__ __device__ constexpr int small_lda(int NQ, int NP) {
  return (NQ * NP > 24 && NQ > 1) ? 16 * NQ + 2 : 16 * NQ + 1;  // (16 NQ + 2) / 2 is odd
}

template <int NQ, int NP, int MQ>
struct Shape {
  // LDA (row stride of A and of Z' / A Li in LDS): NPAD + 1 on the two-wave
  // shapes (their LDS is tight); on the others NPAD + 2 = 2 x odd, where the
  // A x / Z't reads of a half-wave (lanes cl, g in {0, 1}: cl LDA + g doubles)
  // hit 32 distinct bank pairs, instead of two lanes per pair at NPAD + 1
  static constexpr int NPAD = 16 * NQ, KP = 4 * NP, MPAD = 16 * MQ,
                       LDA = small_lda(NQ, NP);
  // k-vector stride KP: lanes read slot 1 / padding elements i >= KP
  // unconditionally and mask the values by their type code (3 = pad), so those
  // reads may alias the next vector (the last one reads into the A block); every
  // write is guarded by i < k or the code, and rows [k, KP) stay zero.
  static constexpr int KS = KP;
  static constexpr int O_RC = O_FIXED;       // rcode[KP]: cone*4 + type (0 POC, 1 SOC head, 2 SOC tail, 3 pad)
  static constexpr int O_KV = O_RC + KP;     // 17 k-vectors, KS apart
  static constexpr int O_A = O_KV + NKV * KS;
  static constexpr int O_NV = O_A + MPAD * LDA;    // n-vectors: c x rd rx n0 tn
  static constexpr int O_MV = O_NV + 6 * NPAD;     // m-vectors: b y rp ry m0 tm
  // U[NCS][NPAD] (the SYRK's cone rows) and, for m <= 16, A Li (MPAD x LDA,
  // from the Schur step to the solves): their lifetimes do not overlap
  static constexpr bool AL_LDS = MQ == 1;
  static constexpr int UAL = (AL_LDS && MPAD * LDA > NCS * NPAD) ? MPAD * LDA : NCS * NPAD;
  static constexpr int O_U = O_MV + 6 * MPAD;
  static constexpr int O_AL = O_U;
  // tile transpose [16][17]: only factor() uses it; on the Cholesky shapes
  // (AL_LDS) in the k-vectors dead during a factorisation when they hold it
  static constexpr bool TB_ALIAS = AL_LDS && NKV_DEAD * KS >= 16 * 17;
  static constexpr int O_TB = TB_ALIAS ? O_KV + KV_RZ * KS : O_U + UAL;
  // the SYRK's U-row table (int32 per k-row) where the LDS allows (not the
  // two-wave shapes, whose LDS is tight)
  static constexpr bool UBT = SOCP_SYRK_UBT && NQ * NP > 24 && NQ > 1;
  static constexpr int O_UBT = O_U + UAL + (TB_ALIAS ? 0 : 16 * 17);
  static constexpr int TOTAL = O_UBT + (UBT ? (KP + 1) / 2 : 0);
  static constexpr int nv(int id) { return O_NV + id * NPAD; }
  static constexpr int mv(int id) { return O_MV + id * MPAD; }
};
enum : int { NV_C, NV_X, NV_RD, NV_RX, NV_N0, NV_TN };
enum : int { MV_B, MV_Y, MV_RP, MV_RY, MV_M0, MV_TM };

// doubles of one factor record of the register kernel: the H^-1 and S^-1
// tiles in lane order, LAM WB CA CBV IL, the per-cone constants, the sing flag
inline int64_t small_rec_doubles(int NQ, int NP, int MQ) {
  const int64_t NT = NQ * (NQ + 1) / 2, MT = MQ * (MQ + 1) / 2;
  const int64_t al = MQ == 1 ? (int64_t)16 * small_lda(NQ, NP) : 0;  // A Li kept in LDS (Shape::AL_LDS)
  return (NT + MT) * 256 + 5 * (int64_t)(4 * NP) + 20 * NCS + al + 8;
}

inline size_t small_lds_bytes(int NQ, int NP, int MQ) {
  int NPAD = 16 * NQ, MPAD = 16 * MQ, LDA = small_lda(NQ, NP);
  int KS = 4 * NP;  // Shape::KS
  int ual = (MQ == 1 && MPAD * LDA > NCS * NPAD) ? MPAD * LDA : NCS * NPAD;  // Shape::UAL
  const bool tb_alias = MQ == 1 && NKV_DEAD * KS >= 16 * 17;                // Shape::TB_ALIAS
  const bool ubt = SOCP_SYRK_UBT && NQ * NP > 24 && NQ > 1;                   // Shape::UBT
  int total = O_FIXED + KS + NKV * KS + MPAD * LDA + 6 * NPAD + 6 * MPAD + ual + (tb_alias ? 0 : 16 * 17) +
              (ubt ? (KS + 1) / 2 : 0);
#ifndef SOCP_DEV_LDS_PAD
#define SOCP_DEV_LDS_PAD 0  // probe builds only: extra LDS bytes per wave to cap the waves per CU
#endif
  return (size_t)total * sizeof(double) + SOCP_DEV_LDS_PAD;
}

// Diagnostic phase timing (separate build, -DSOCP_DIAG): per-phase s_memtime
// deltas accumulated per problem and added to a global table by lane 0.
#ifdef SOCP_DIAG
#define NSTAMP 12
#define NSUBSTAMP 11  // sub-phases (0-3 the H sweep, 4-10 solve / cone-op parts), slots NSTAMP+1 ..
// Totals live in LDS (lane 0 read-modify-writes them), so the stamps cost no
// registers beyond the last timestamp; they are flushed once per wave.
#define STAMP_DECL uint64_t st_last = 0;
#define STAMP_START_S(obj) do { __builtin_amdgcn_s_waitcnt(0); (obj).st_last = __builtin_amdgcn_s_memtime(); } while (0)
#define STAMP(i) do { __builtin_amdgcn_s_waitcnt(0); const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    if (threadIdx.x == 0) reinterpret_cast<unsigned long long*>(socp_lds + O_STAMPS)[i] += t_ - st_last; \
    st_last = t_; } while (0)
#define STAMP_SUB(i) do { if constexpr (SUBST) STAMP(NSTAMP + 1 + (i)); } while (0)
#define STAMP_X(i) STAMP(NSTAMP + 1 + (i))
#else
#define STAMP_DECL
#define STAMP_START_S(obj) do {} while (0)
#define STAMP(i) do {} while (0)
#define STAMP_SUB(i) do {} while (0)
#define STAMP_X(i) do {} while (0)
#endif
enum { SP_LOAD, SP_SCALING, SP_RESID, SP_U, SP_SYRK, SP_SWEEP_H, SP_SCHUR, SP_SOLVE, SP_STEP, SP_VOP,
       SP_STORE, SP_OTHER };

// Static-analysis build (-DSOCP_MARK, tools/isa_phases.py): region markers as
// assembly comments; never in a product or diagnostic library.
#ifdef SOCP_MARK
#define MARK_BEGIN(name) asm volatile(";@@BEGIN " name)
#define MARK_END(name) asm volatile(";@@END " name)
#else
#define MARK_BEGIN(name) do {} while (0)
#define MARK_END(name) do {} while (0)
#endif

extern __shared__ double socp_lds[];
#define LDS(i) socp_lds[(i)]
// Blocks are one wavefront: LDS instructions of a wave execute in issue order,
// so an LDS hand-off between lanes needs only a wave-scope fence (no s_barrier,
// no lgkmcnt drain) -- the rocPRIM wave_barrier() idiom.
#define SYNC()                                             \
  do {                                                     \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); \
    __builtin_amdgcn_wave_barrier();                       \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); \
  } while (0)

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

// A row step of G (NQ doubles) out of its AGPRs in ONE asm statement: the
// compiler pads one wait state after an asm that defines a VGPR a VALU op
// reads next, so reading the row together pays it once per row, not per value.
template <int NQ>
__device__ __forceinline__ void a_get_row(const AD (&r)[NQ], double (&out)[NQ]) {
  uint32_t lo[4], hi[4];
  if constexpr (NQ == 1) {
    asm("v_accvgpr_read_b32 %0, %2\n\tv_accvgpr_read_b32 %1, %3" : "=v"(lo[0]), "=v"(hi[0]) : "a"(r[0].lo), "a"(r[0].hi));
  } else if constexpr (NQ == 2) {
    asm("v_accvgpr_read_b32 %0, %4\n\tv_accvgpr_read_b32 %1, %5\n\tv_accvgpr_read_b32 %2, %6\n\t"
        "v_accvgpr_read_b32 %3, %7"
        : "=v"(lo[0]), "=v"(hi[0]), "=v"(lo[1]), "=v"(hi[1])
        : "a"(r[0].lo), "a"(r[0].hi), "a"(r[1].lo), "a"(r[1].hi));
  } else if constexpr (NQ == 3) {
    asm("v_accvgpr_read_b32 %0, %6\n\tv_accvgpr_read_b32 %1, %7\n\tv_accvgpr_read_b32 %2, %8\n\t"
        "v_accvgpr_read_b32 %3, %9\n\tv_accvgpr_read_b32 %4, %10\n\tv_accvgpr_read_b32 %5, %11"
        : "=v"(lo[0]), "=v"(hi[0]), "=v"(lo[1]), "=v"(hi[1]), "=v"(lo[2]), "=v"(hi[2])
        : "a"(r[0].lo), "a"(r[0].hi), "a"(r[1].lo), "a"(r[1].hi), "a"(r[2].lo), "a"(r[2].hi));
  } else {
    static_assert(NQ == 4, "NQ <= 4");
    asm("v_accvgpr_read_b32 %0, %8\n\tv_accvgpr_read_b32 %1, %9\n\tv_accvgpr_read_b32 %2, %10\n\t"
        "v_accvgpr_read_b32 %3, %11\n\tv_accvgpr_read_b32 %4, %12\n\tv_accvgpr_read_b32 %5, %13\n\t"
        "v_accvgpr_read_b32 %6, %14\n\tv_accvgpr_read_b32 %7, %15"
        : "=v"(lo[0]), "=v"(hi[0]), "=v"(lo[1]), "=v"(hi[1]), "=v"(lo[2]), "=v"(hi[2]), "=v"(lo[3]), "=v"(hi[3])
        : "a"(r[0].lo), "a"(r[0].hi), "a"(r[1].lo), "a"(r[1].hi), "a"(r[2].lo), "a"(r[2].hi), "a"(r[3].lo),
          "a"(r[3].hi));
  }
#pragma unroll
  for (int q = 0; q < NQ; ++q) out[q] = __longlong_as_double((long long)(((uint64_t)hi[q] << 32) | lo[q]));
}

// a_get for a value consumed directly as an MFMA A/B operand: v_accvgpr_read is
// a VALU write, and VALU write -> MFMA operand read needs 2 wait states, which
// hipcc does not insert for a producer inside inline asm (it pads one state).
__device__ __forceinline__ double a_get_mfma(const AD& r) {
  uint32_t lo, hi;
  asm("v_accvgpr_read_b32 %0, %2\n\tv_accvgpr_read_b32 %1, %3\n\ts_nop 1"
      : "=v"(lo), "=v"(hi)
      : "a"(r.lo), "a"(r.hi));
  return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Scheduling fence: keeps the scheduler from hoisting the next unrolled step's
// loads above this point (with H pinned in VGPRs and G in AGPRs, hoisting
// across steps is what overflows the register file).
#define SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ constexpr int tri(int i, int j) { return i * (i + 1) / 2 + j; }
__device__ __forceinline__ double sel4(d4 t, int r) {
  double v = t[0];
  v = (r == 1) ? t[1] : v;
  v = (r == 2) ? t[2] : v;
  v = (r == 3) ? t[3] : v;
  return v;
}

// DPP move of a double (two 32-bit halves).  CTRL: 0x111+s = row_shr:s+1,
// 0x142 = row_bcast:15, 0x143 = row_bcast:31 (GFX9 DPP); RM = row mask.
template <int CTRL, int RM>
__device__ __forceinline__ double dpp(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int l2 = __builtin_amdgcn_update_dpp(0, lo, CTRL, RM, 0xF, false);
  const int h2 = __builtin_amdgcn_update_dpp(0, hi, CTRL, RM, 0xF, false);
  return __hiloint2double(h2, l2);
}
// DPP move whose pattern writes every lane (row_newbcast): no old value needed.
template <int CTRL>
__device__ __forceinline__ double dpp_all(double v) {
  const int l2 = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
  const int h2 = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
  return __hiloint2double(h2, l2);
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// Lane ids re-read inside each phase (LANE_IDS shadows the members): values
// derived from them (4*pp + g, 16*ti + cl, ...) are then recomputed where they
// are used instead of being hoisted out of the persistent loop and kept live.
#ifndef SOCP_MULTI_WAVE
#define SOCP_MULTI_WAVE 0  // 1: workgroups of several wavefronts (socp_large.hip defines it)
#endif
__device__ __forceinline__ int lane_fresh() {
  int v = SOCP_MULTI_WAVE ? (int)threadIdx.x & 63 : (int)threadIdx.x;  // the lane in its wavefront
  asm volatile("" : "+v"(v));
  return v;
}
#define LANE_IDS()                      \
  const int lane = lane_fresh();        \
  const int g = lane >> 4, cl = lane & 15; \
  (void)g; (void)cl

// Sum over the four 16-lane rows (lanes l, l^16, l^32, l^48) with the gfx950
// row-swap permutes: every lane gets the same total, no LDS round trip.
__device__ __forceinline__ double rows_sum(double x) {
  const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
  const auto a = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  const double y = __hiloint2double((int)b[0], (int)a[0]) + __hiloint2double((int)b[1], (int)a[1]);
  const unsigned ylo = (unsigned)__double2loint(y), yhi = (unsigned)__double2hiint(y);
  const auto c = __builtin_amdgcn_permlane16_swap(ylo, ylo, false, false);
  const auto d = __builtin_amdgcn_permlane16_swap(yhi, yhi, false, false);
  return __hiloint2double((int)d[0], (int)c[0]) + __hiloint2double((int)d[1], (int)c[1]);
}

// Cone reductions when every cone is R = 1, 2 or 4 whole 16-lane rows (all
// cones 16, 32 or 64 long): all-reduce inside each row by DPP rotations, then
// across the cone's rows with the row-swap permutes -- every lane of the cone
// gets the total, no predicates, no LDS.  MX: max instead of sum.
template <bool MX>
__device__ __forceinline__ double rop(double a, double b) { return MX ? fmax(a, b) : a + b; }
// Several independent values at once, step by step (each DPP step of one
// chain waits on its predecessor; interleaving the chains fills those wait
// states).  The same operations in the same order per value as
// cone_allreduce_rows.  MXM: bit q set = max for value q.
template <int NV, unsigned MXM>
__device__ __forceinline__ void cone_allreduce_rows_n(double (&v)[NV], int R) {
#define SOCP_AR_STEP(CTRL)                                                                          \
  _Pragma("unroll") for (int q = 0; q < NV; ++q) {                                                  \
    const double y = dpp_all<CTRL>(v[q]);                                                           \
    v[q] = ((MXM >> q) & 1) ? fmax(v[q], y) : v[q] + y;                                             \
  }
  SOCP_AR_STEP(0x128)
  SOCP_AR_STEP(0x124)
  SOCP_AR_STEP(0x122)
  SOCP_AR_STEP(0x121)
#undef SOCP_AR_STEP
  if (R >= 2) {
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const unsigned lo = (unsigned)__double2loint(v[q]), hi = (unsigned)__double2hiint(v[q]);
      const auto c = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
      const auto d = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
      const double a = __hiloint2double((int)d[0], (int)c[0]), b = __hiloint2double((int)d[1], (int)c[1]);
      v[q] = ((MXM >> q) & 1) ? fmax(a, b) : a + b;
    }
  }
  if (R == 4) {
#pragma unroll
    for (int q = 0; q < NV; ++q) {
      const unsigned lo = (unsigned)__double2loint(v[q]), hi = (unsigned)__double2hiint(v[q]);
      const auto c = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
      const auto d = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
      const double a = __hiloint2double((int)d[0], (int)c[0]), b = __hiloint2double((int)d[1], (int)c[1]);
      v[q] = ((MXM >> q) & 1) ? fmax(a, b) : a + b;
    }
  }
}
template <bool MX>
__device__ __forceinline__ double cone_allreduce_rows(double v, int R) {
  v = rop<MX>(v, dpp_all<0x128>(v));  // row_ror:8
  v = rop<MX>(v, dpp_all<0x124>(v));  // row_ror:4
  v = rop<MX>(v, dpp_all<0x122>(v));  // row_ror:2
  v = rop<MX>(v, dpp_all<0x121>(v));  // row_ror:1
  if (R >= 2) {  // rows (2r, 2r+1)
    const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
    const auto c = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto d = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    v = rop<MX>(__hiloint2double((int)d[0], (int)c[0]), __hiloint2double((int)d[1], (int)c[1]));
  }
  if (R == 4) {  // halves (l, l ^ 32)
    const unsigned lo = (unsigned)__double2loint(v), hi = (unsigned)__double2hiint(v);
    const auto c = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto d = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    v = rop<MX>(__hiloint2double((int)d[0], (int)c[0]), __hiloint2double((int)d[1], (int)c[1]));
  }
  return v;
}

// Butterfly partner inside a 16-lane row for reduce-scatter level M, by DPP:
// M=8 row_ror:8 (l^8), M=4 row_half_mirror (l^7: flips bit 2 like l^4, so the
// halving is the same), M=2 quad_perm[2,3,0,1] (l^2), M=1 quad_perm[1,0,3,2].
template <int M>
__device__ __forceinline__ double row_partner(double v) {
  constexpr int CTRL = M == 8 ? 0x128 : (M == 4 ? 0x141 : (M == 2 ? 0x4E : 0xB1));
  return dpp_all<CTRL>(v);
}

// Wave-uniform copies.  LLVM's divergence analysis treats every LDS or global
// load as divergent; a branch on such a value (the sweep's pivot test, the
// per-problem `sing` flag, the phase number) is then compiled as exec-masked
// straight-line code: every arm runs and the live ranges of all arms merge.
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ double uni(double v) {
  const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
  const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
  return __hiloint2double(hi, lo);
}

// Inclusive segmented scan over the 64 lanes with DPP (row_shr 1,2,4,8 then
// row_bcast 15/31): lane l accumulates lanes [max(ssl, 0) .. l] with op
// (sum, or max when mx).  ssl = first lane of l's segment.
template <int V>
__device__ __forceinline__ void dpp_scan(double (&x)[V], int lane, int ssl, bool mx) {
  const int rl = lane & 15;
#define SOCP_SCAN_STEP(CTRL, RM, OK)                                 \
  {                                                                  \
    const bool ok_ = (OK);                                           \
    _Pragma("unroll") for (int v = 0; v < V; ++v) {                  \
      const double y = dpp<CTRL, RM>(x[v]);                          \
      const double r = mx ? fmax(x[v], y) : x[v] + y;                \
      x[v] = ok_ ? r : x[v];                                         \
    }                                                                \
  }
  SOCP_SCAN_STEP(0x111, 0xF, rl >= 1 && lane - 1 >= ssl)
  SOCP_SCAN_STEP(0x112, 0xF, rl >= 2 && lane - 2 >= ssl)
  SOCP_SCAN_STEP(0x114, 0xF, rl >= 4 && lane - 4 >= ssl)
  SOCP_SCAN_STEP(0x118, 0xF, rl >= 8 && lane - 8 >= ssl)
  SOCP_SCAN_STEP(0x142, 0xA, ((lane >> 4) & 1) && ((lane & ~15) - 1 >= ssl))
  SOCP_SCAN_STEP(0x143, 0xC, lane >= 32 && 31 >= ssl)
#undef SOCP_SCAN_STEP
}

// whole-wave sum / max (scan to lane 63, broadcast through an SGPR)
__device__ __forceinline__ double wsum(double v) {
  double x[1] = {v};
  dpp_scan<1>(x, threadIdx.x, 0, false);
  return readlane_d(x[0], 63);
}
__device__ __forceinline__ double wmax(double v) {
  double x[1] = {v};
  dpp_scan<1>(x, threadIdx.x, 0, true);
  return readlane_d(x[0], 63);
}

// x^e for an integer exponent (Julia's ^(::Float64, ::Integer); e = 3 is x*x*x)
__device__ __forceinline__ double ipow(double x, int e) {
  if (e == 3) return x * x * x;
  double r = 1.0, b = x;
  for (int q = e; q > 0; q >>= 1) {
    if (q & 1) r *= b;
    b *= b;
  }
  return r;
}

// IEEE classes (v_cmp_class_f64 mask bits) at which the Newton refinement of
// a v_rcp / v_rsq seed would turn an exact 0 or inf into NaN (0 * inf): +-0,
// +-inf.  There the seed is the IEEE result itself and is returned as is.
constexpr int kClassZeroInf = (1 << 2) | (1 << 5) | (1 << 6) | (1 << 9);

// pivot reciprocal: v_rcp_f64 + two Newton steps (within 1 ulp of 1/d; 1/+-0 =
// +-inf and 1/+-inf = +-0 exactly, as IEEE division gives)
__device__ __forceinline__ double recip(double d) {
  const double r0 = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r0, 1.0);
  double r = fma(r0, e, r0);
  e = fma(-d, r, 1.0);
  r = fma(r, e, r);
  return __builtin_amdgcn_class(d, kClassZeroInf) ? r0 : r;
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
      P[j] = mine + row_partner<M>(other);
    }
    if (hi) base += H;
    rs16<H, M / 2>(P, cl, base);
  } else {
#pragma unroll
    for (int j = 0; j < C; ++j) P[j] += row_partner<M>(P[j]);
    rs16<C, M / 2>(P, cl, base);
  }
}
// the lane's first entry index after rs16<C, M> (its `base`), known up front
template <int C, int M>
__device__ __forceinline__ int rs16_base(int cl) {
  if constexpr (M == 0) {
    return 0;
  } else if constexpr (C % 2 == 0) {
    return ((cl & M) != 0 ? C / 2 : 0) + rs16_base<C / 2, M / 2>(cl);
  } else {
    return rs16_base<C, M / 2>(cl);
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

// driver micro-phases and solve kinds
enum : int {
  MP_SINGTEST, MP_SINGTEST_POST, MP_FACTOR, MP_INIT, MP_ITER, MP_KKT,
  MP_SOLVE_HEAD, MP_SOLVE_MAT, MP_SOLVE_TAIL, MP_SAVE
};
enum : int { RET_INIT, RET_KKT, RET_AFFINE, RET_COMBINED };

// ---------------------------------------- 16x16 tile kernels (shared by the
// register kernel's H^-1 sweep and the blocked kernel's panel factorisation)

// Broadcast across the four 16-lane rows: every lane gets x from the lane of
// row R with the same column index (gfx950 v_permlane32_swap / 16_swap).
template <int R>
__device__ __forceinline__ double row_bcast(double x) {
  const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
  const auto a32 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b32 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  const unsigned ylo = (R < 2) ? a32[0] : a32[1], yhi = (R < 2) ? b32[0] : b32[1];
  const auto a16 = __builtin_amdgcn_permlane16_swap(ylo, ylo, false, false);
  const auto b16 = __builtin_amdgcn_permlane16_swap(yhi, yhi, false, false);
  const unsigned zlo = (R & 1) ? a16[1] : a16[0], zhi = (R & 1) ? b16[1] : b16[0];
  return __hiloint2double((int)zhi, (int)zlo);
}

// All four row broadcasts of x at once: out[R] = x of row R, same column index.
__device__ __forceinline__ void row_bcast4(double x, double (&out)[4]) {
  const unsigned lo = (unsigned)__double2loint(x), hi = (unsigned)__double2hiint(x);
  const auto a32 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto b32 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const auto a16 = __builtin_amdgcn_permlane16_swap(a32[h], a32[h], false, false);
    const auto b16 = __builtin_amdgcn_permlane16_swap(b32[h], b32[h], false, false);
    out[2 * h] = __hiloint2double((int)b16[0], (int)a16[0]);
    out[2 * h + 1] = __hiloint2double((int)b16[1], (int)a16[1]);
  }
}

// x^-1/2: v_rsq_f64 + two Newton steps (within 1 ulp; +-0 -> +-inf and
// +inf -> 0 as 1/sqrt gives them in IEEE arithmetic, negative -> NaN)
__device__ __forceinline__ double rsqrt_nr(double d) {
  const double y0 = __builtin_amdgcn_rsq(d);
  const double h = 0.5 * d;
  double e = fma(-(h * y0), y0, 0.5);
  double y = fma(y0, e, y0);
  e = fma(-(h * y), y, 0.5);
  y = fma(y, e, y);
  return __builtin_amdgcn_class(d, kClassZeroInf) ? y0 : y;
}
// x * q for q = rsqrt_nr(p) where p = 0 makes q = inf: an exact zero factor
// stays zero, as sqrt(0 * y) and sqrt(0 / y) are in IEEE arithmetic (a
// boundary iterate of a POC cone, s_i z_i = 0), instead of 0 * inf = NaN
__device__ __forceinline__ double zmul(double x, double q) { return x == 0.0 ? x : x * q; }
// square root through rsqrt_nr (0 and +inf passed through, negative -> NaN)
__device__ __forceinline__ double sqrt_nr(double d) {
  const double r = d * rsqrt_nr(d);
  return (d == 0.0 || d == INFINITY) ? d : r;
}
// the tile factorisation's pivots: SOCP_TILE_NEWTON Newton steps (1: a
// shorter dependency chain, within a few ulp)
#ifndef SOCP_TILE_NEWTON
#define SOCP_TILE_NEWTON 1
#endif
__device__ __forceinline__ double rsqrt_tile(double d) {
#if SOCP_TILE_NEWTON == 1
  const double y = __builtin_amdgcn_rsq(d);
  const double e = fma(-(0.5 * d) * y, y, 0.5);
  return fma(y, e, y);
#else
  return rsqrt_nr(d);
#endif
}

#ifndef SOCP_TILE_FACTOR
#define SOCP_TILE_FACTOR 1
#endif
#ifndef SOCP_TRANSPOSE_MFMA
#define SOCP_TRANSPOSE_MFMA 0
#endif
#ifndef SOCP_U_LANECONES
#define SOCP_U_LANECONES 1  // compute_U takes the cone descriptors from the cone lanes (0: from the kernel args)
#endif
#ifndef SOCP_TILE_OKDIAG
#define SOCP_TILE_OKDIAG 1  // the pivot test once per tile, on the diagonal of W (0: per pivot)
#endif
#ifndef SOCP_S_TILE
#define SOCP_S_TILE 1  // m <= 16 Cholesky shapes: S^-1 = W'W from one factor_tile (0: Gauss-Jordan sweep)
#endif
#ifndef SOCP_TILE_INPLACE
#define SOCP_TILE_INPLACE 1  // 0: copy back only registers > B (A/B builds)
#endif
#if SOCP_TILE_FACTOR == 0
// Pivot J of row block B of the tile factorisation: v = register B of the
// (updated) D tile, w = register B of the eliminated identity.  Row J of
// the block (lanes of row group J) is scaled by 1/sqrt(d) and becomes row
// 4B+J of L' (R) and of W; the rows below it in the block take the rank-1
// update.  Rows above it (finished) take garbage, never read again.
template <int B, int J>
__device__ __forceinline__ void tile_pivot(double& v, double& w, double& R, double& Wb, bool& ok) {
  if constexpr (J < 4) {
    LANE_IDS();
    const double d = readlane_d(v, 16 * J + 4 * B + J);
    ok = ok && (d > 0.0);  // NaN fails too: potrf's test
    const double rs = rsqrt_nr(d);
    const double vj = row_bcast<J>(v) * rs;
    const double wj = row_bcast<J>(w) * rs;
    const double l = dpp_all<0x150 + 4 * B + J>(v) * rs;  // D[4B+g][4B+J] / sqrt(d)
    v = fma(-l, vj, v);
    w = fma(-l, wj, w);
    R = (g == J) ? vj : R;
    Wb = (g == J) ? wj : Wb;
    tile_pivot<B, J + 1>(v, w, R, Wb, ok);
  }
}
#endif
// Row blocks B.. of W = L^-1 for D = L L' (right-looking, 4 rows at a time;
// the rank-4 trailing update of the D and identity tiles is one MFMA each).
// The 4x4 diagonal block is factored in wave-uniform values (its upper
// triangle, as potrf('U') reads it), then every lane forms the block's rows
// of R = L' and of W by forward substitution from the broadcast block rows.
struct NoHook {
  template <int B>
  __device__ __forceinline__ void run() const {}
};
template <int B, bool INPL = (SOCP_TILE_INPLACE != 0), class H = NoHook>
__device__ __forceinline__ void tile_block(d4& Dt, d4& It, d4& W, bool& ok, const H& hook = H()) {
  if constexpr (B < 4) {
    LANE_IDS();
    double R, Wb;
#if SOCP_TILE_FACTOR == 0
    {
      double v = Dt[B], w = It[B];
      R = 0.0;
      Wb = 0.0;
      tile_pivot<B, 0>(v, w, R, Wb, ok);
    }
#else
    {
      const double v = Dt[B], w = It[B];
      // a_ij = D[4B+i][4B+j] (i <= j): lane (i, 4B+j) of register B
      const double a00 = readlane_d(v, 4 * B), a01 = readlane_d(v, 4 * B + 1),
                   a02 = readlane_d(v, 4 * B + 2), a03 = readlane_d(v, 4 * B + 3);
      const double a11 = readlane_d(v, 16 + 4 * B + 1), a12 = readlane_d(v, 16 + 4 * B + 2),
                   a13 = readlane_d(v, 16 + 4 * B + 3);
      const double a22 = readlane_d(v, 32 + 4 * B + 2), a23 = readlane_d(v, 32 + 4 * B + 3);
      const double a33 = readlane_d(v, 48 + 4 * B + 3);
      const double rs0 = rsqrt_tile(a00);
      const double r01 = a01 * rs0, r02 = a02 * rs0, r03 = a03 * rs0;
      const double s11 = fma(-r01, r01, a11);
      const double rs1 = rsqrt_tile(s11);
      const double r12 = fma(-r01, r02, a12) * rs1, r13 = fma(-r01, r03, a13) * rs1;
      const double s22 = fma(-r12, r12, fma(-r02, r02, a22));
      const double rs2 = rsqrt_tile(s22);
      const double r23 = fma(-r12, r13, fma(-r02, r03, a23)) * rs2;
      const double s33 = fma(-r23, r23, fma(-r13, r13, fma(-r03, r03, a33)));
      const double rs3 = rsqrt_tile(s33);
#if !SOCP_TILE_OKDIAG
      ok = ok && (a00 > 0.0) && (s11 > 0.0) && (s22 > 0.0) && (s33 > 0.0);  // NaN fails too
#endif
      double V[4], X[4];
      row_bcast4(v, V);
      row_bcast4(w, X);
      const double R0 = V[0] * rs0;
      const double R1 = fma(-r01, R0, V[1]) * rs1;
      const double R2 = fma(-r12, R1, fma(-r02, R0, V[2])) * rs2;
      const double R3 = fma(-r23, R2, fma(-r13, R1, fma(-r03, R0, V[3]))) * rs3;
      const double W0 = X[0] * rs0;
      const double W1 = fma(-r01, W0, X[1]) * rs1;
      const double W2 = fma(-r12, W1, fma(-r02, W0, X[2])) * rs2;
      const double W3 = fma(-r23, W2, fma(-r13, W1, fma(-r03, W0, X[3]))) * rs3;
      R = g == 0 ? R0 : (g == 1 ? R1 : (g == 2 ? R2 : R3));
      Wb = g == 0 ? W0 : (g == 1 ? W1 : (g == 2 ? W2 : W3));
    }
#endif
    hook.template run<B>();  // independent MFMA work interleaved with the chain
    W[B] = Wb;
    if constexpr (B < 3 && INPL) {
      // whole tiles: registers <= B are never read again (the later blocks read
      // registers B+1..3), so the MFMA results replace Dt and It in place
      Dt = __builtin_amdgcn_mfma_f64_16x16x4f64(R, R, Dt, 0, 0, 1);   // Dt -= R'R
      It = __builtin_amdgcn_mfma_f64_16x16x4f64(R, Wb, It, 0, 0, 1);  // It -= R'W
    } else if constexpr (B < 3) {
      const d4 t = __builtin_amdgcn_mfma_f64_16x16x4f64(R, R, Dt, 0, 0, 1);   // Dt -= R'R
      const d4 u = __builtin_amdgcn_mfma_f64_16x16x4f64(R, Wb, It, 0, 0, 1);  // It -= R'W
#pragma unroll
      for (int r = B + 1; r < 4; ++r) {
        Dt[r] = t[r];
        It[r] = u[r];
      }
    }
    tile_block<B + 1, INPL>(Dt, It, W, ok, hook);
  }
}
// INPL: the trailing updates replace the tiles whole (one factorisation 3,126
// cycles vs 3,406 on one wave, profiles/r03_probe_tile.log); the copying form
// keeps fewer registers live, which the smallest register kernels need to stay
// at two waves per SIMD.
template <bool INPL = (SOCP_TILE_INPLACE != 0), class H = NoHook>
__device__ __forceinline__ void factor_tile(d4 Dt, d4& W, bool& ok, const H& hook = H()) {
  MARK_BEGIN("factor_tile");
  LANE_IDS();
  d4 It;
#pragma unroll
  for (int r = 0; r < 4; ++r) It[r] = (g + 4 * r == cl) ? 1.0 : 0.0;
  W = It;
  tile_block<0, INPL>(Dt, It, W, ok, hook);
#if SOCP_TILE_OKDIAG
  // potrf's test once per tile: the diagonal of W = L^-1 holds the pivots'
  // 1/sqrt, which is finite and > 0 exactly when every pivot is > 0 (a pivot
  // <= 0 or NaN makes rsqrt_tile NaN; a NaN anywhere reaches every later pivot)
  bool dg = true;
#pragma unroll
  for (int r = 0; r < 4; ++r) dg = dg && (g + 4 * r != cl || W[r] > 0.0);
  ok = ok && __all(dg);
#endif
}


// XI (SOCP_F_EXPLICIT_INVERSE): Li = H^-1 formed on every shape -- the
// reference's operation order (densesolver.jl:47-48 forms Li = L^-T L^-1 from
// cholesky!(H)) -- instead of the triangular solves of the m <= 16 shapes.
template <int NQ, int NP, int MQ, bool XI = false>
struct Small {
  using SH = Shape<NQ, NP, MQ>;
  static constexpr int NT = NQ * (NQ + 1) / 2;
  static constexpr int MT = MQ * (MQ + 1) / 2;
  static constexpr int NPAD = SH::NPAD, KP = SH::KP, MPAD = SH::MPAD, LDA = SH::LDA;
  static constexpr int O_A = SH::O_A, O_U = SH::O_U, O_AL = SH::O_AL, O_TB = SH::O_TB, O_RC = SH::O_RC,
                       O_KV = SH::O_KV;
  static constexpr bool AL_LDS = SH::AL_LDS;
  // in-place tile updates (factor_tile) except where G is small enough for two
  // waves per SIMD: C1's <2, 12, 1> takes 209 + 48 registers with them, 208 + 48
  // without
  static constexpr bool TILE_INPL = SOCP_TILE_INPLACE != 0 && NQ * NP > 24;
  // the solves' per-cone constants read ahead of the cone reductions (their
  // latency under the DPP chains) where registers allow: not in the kernels
  // that keep two waves per SIMD (C1's <2, 12, 1> would take 217 + 48; every
  // NQ = 1 shape)
  static constexpr bool HOIST_CST = NQ * NP > 24 && NQ > 1;
  static constexpr int C_ = SH::nv(NV_C), X_ = SH::nv(NV_X), RD = SH::nv(NV_RD),
                       RX = SH::nv(NV_RX), N0 = SH::nv(NV_N0), TN = SH::nv(NV_TN);
  static constexpr int B_ = SH::mv(MV_B), Y_ = SH::mv(MV_Y), RP = SH::mv(MV_RP),
                       RY = SH::mv(MV_RY), M0 = SH::mv(MV_M0);
  static constexpr int kvs(int id) { return O_KV + id * SH::KS; }
  static constexpr int H_ = kvs(KV_H), Z_ = kvs(KV_Z), S_ = kvs(KV_S), DZ = kvs(KV_DZ),
                       DS = kvs(KV_DS), RZ = kvs(KV_RZ), RS = kvs(KV_RS), LAM = kvs(KV_LAM),
                       WB = kvs(KV_WB), CA = kvs(KV_CA), CBV = kvs(KV_CB), K0 = kvs(KV_K0),
                       K1 = kvs(KV_K1), K2 = kvs(KV_K2), T1 = kvs(KV_T1), T2 = kvs(KV_T2),
                       IL = kvs(KV_IL);

  const SmallArgs& a;
  const int lane, g, cl;
  const int n, m, k, nc;
  bool sing;
  int64_t dbg_p = 0;
  // compact-layout element info (element i = 64*s + lane): cone, type code
  // (0 POC, 1 SOC head, 2 SOC tail, 3 none), cone offset, scan segment
  // start / last lane within the slot
  int ci[2], kd[2], eo[2], ssl[2], sle[2];
  bool spn[2];  // the lane's cone spans both slots
  STAMP_DECL

  AD G[NP][NQ];  // AGPR-resident
  d4 T[NT];
  d4 Sv[MT];
#ifndef SOCP_KEEP_AL
#define SOCP_KEEP_AL 0
#endif
  // A Li (m x n) as C/D tiles AL[tq][ti] = (A Li)[16tq.., 16ti..]: kept from
  // the Schur step for the solves' cx = Li n0 + (A Li)' m0 (shapes with at
  // most 4 such tiles; larger ones take A'm0 and a second Li product)
  static constexpr bool KEEP_AL = SOCP_KEEP_AL && NQ * MQ <= 4;
  d4 AL[KEEP_AL ? MQ : 1][KEEP_AL ? NQ : 1];
#ifndef SOCP_SMALL_CHOL
#define SOCP_SMALL_CHOL 1  // 0: Li = H^-1 by the Gauss-Jordan sweep for every shape (A/B builds)
#endif
  // m <= 16: H = L L' (chol), Z = L^-1 A' in LDS, S = Z'Z; Li is never formed
  // and its products are triangular solves (trsv_fwd / trsv_bwd).  Larger m
  // keep the explicit inverse by the sweep.
  static constexpr bool CHOL = SOCP_SMALL_CHOL && AL_LDS && !KEEP_AL && !XI;
#ifndef SOCP_INV_CHOL
#define SOCP_INV_CHOL 1  // 0: the explicit inverses by the Gauss-Jordan sweep (A/B builds)
#endif
  // where Li = H^-1 is formed (XI; the m > 16 shapes): from the Cholesky
  // factor, Li = L^-T L^-1 (densesolver.jl:47-48, chol_inv), and likewise
  // S^-1; the SYRK then leaves H in the upper-block form chol() reads
  static constexpr bool INV_CHOL = SOCP_INV_CHOL && !CHOL;
  static constexpr bool UPPER_H = CHOL || INV_CHOL;

  __device__ __forceinline__ Small(const SmallArgs& args)
      : a(args), lane(threadIdx.x), g(threadIdx.x >> 4), cl(threadIdx.x & 15),
        n(args.n), m(args.m), k(args.k), nc(args.nc) {}

  // ---------------------------------------------------------------- setup
  // O_U + cone(row) * NPAD per k-row (int32, launch-wide: the cone table is
  // the batch's), for the SYRK's U rows (SOCP_SYRK_UBT shapes)
  __device__ __forceinline__ int ubt(int row) const { return reinterpret_cast<const int*>(socp_lds + SH::O_UBT)[row]; }
  __device__ __forceinline__ void init_tables() {
    if (lane < nc) {
      LDS(O_COFF + lane) = a.cones.offs[lane];
      LDS(O_CDIM + lane) = a.cones.dim[lane];
      LDS(O_CKIND + lane) = a.cones.kind[lane];
      if constexpr (HOIST_CST) {
        lc_soc = a.cones.kind[lane] == SOC_K;
        lc_off = a.cones.offs[lane];
        lc_dim = a.cones.dim[lane];
      }
    }
    for (int i = lane; i < KP; i += 64) {
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
      if constexpr (SH::UBT) reinterpret_cast<int*>(socp_lds + SH::O_UBT)[i] = O_U + (code >> 2) * NPAD;
    }
    // segment partials: entry (v, c, slot) is written only when cone c meets the
    // slot, the same for every problem of the launch; the rest stays zero
    for (int e = lane; e < O_TOTC - O_PART; e += 64) LDS(O_PART + e) = 0.0;
#ifdef SOCP_DIAG
    if (lane < 24) LDS(O_STAMPS + lane) = 0.0;  // all-zero bits: the u64 totals start at 0
#endif
    SYNC();
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = 64 * s + lane;
      const bool ev = i < k;
      const int code = ev ? (int)LDS(O_RC + i) : 3;
      const int c = ev ? (code >> 2) : 0;
      ci[s] = c;
      kd[s] = ev ? (code & 3) : 3;
      const int o = ev ? (int)LDS(O_COFF + c) : i;
      const int d = ev ? (int)LDS(O_CDIM + c) : 1;
      eo[s] = o;
      const int st = o > 64 * s ? o : 64 * s;
      const int en = (o + d) < 64 * (s + 1) ? (o + d) : 64 * (s + 1);
      spn[s] = ev && o < 64 && o + d > 64;
      ssl[s] = ev ? st - 64 * s : lane;
      sle[s] = ev ? en - 1 - 64 * s : -1;
    }
  }

#ifndef SOCP_KO
#define SOCP_KO 0  // timing knock-outs (tuning builds only; results are wrong): 1 G loaded once per wave,
                   // 2 no residuals, 4 no compute_U, 8 no S factorisation, 16 no Gx, 32 no G'z (residuals),
                   // 128 no A products (residuals), 256 no triangular solves, 512 / 1024 no G products
                   // in the solves, 2048 no S solves, 4096 no scaling, 8192 no solve head,
                   // 16384 no solve tail, 32768 no corrector, 65536 no SYRK (H = I), 131072 no chol
#endif
  bool ko_gloaded = false;
  // lane c < nc: its cone's kind and offset (per-cone work without the table
  // round trips)
  bool lc_soc = false;
  int lc_off = 0, lc_dim = 0;
  __device__ __forceinline__ void load_problem(int64_t p) {
    MARK_BEGIN("load_problem");
    LANE_IDS();
    const double* Gp = a.G + p * (int64_t)k * n;
    // the vectors and the first chunk of A are requested first: their HBM
    // round trip runs under G's (n, m <= 64 here, k <= 128)
    const double cv = lane < n ? a.c[p * n + lane] : 0.0;
    const double bv = lane < m ? a.b[p * m + lane] : 0.0;
    const double hv0 = lane < k ? a.h[p * k + lane] : 0.0;
    const double hv1 = lane + 64 < k ? a.h[p * k + 64 + lane] : 0.0;
    const double* Ap = a.A + p * (int64_t)m * n;
    const int mn = m * n;
    constexpr int AB = HOIST_CST ? 16 : 8;
    double av[AB];
#pragma unroll
    for (int t = 0; t < AB; ++t) av[t] = (64 * t + lane < mn) ? Ap[64 * t + lane] : 0.0;
    if (!(SOCP_KO & 1) || !ko_gloaded) {
    ko_gloaded = true;
    // G -> AGPRs.  a_put is an asm statement the scheduler does not move loads
    // across, so the loads are issued in batches of 16 into VGPRs first (one
    // HBM round trip per batch, not per element).  Raw buffer loads over the
    // problem's G (k n doubles): a padding element (row >= k or col >= n)
    // takes an offset past the range and reads 0 -- no address arithmetic in
    // 64 bits, no branch, no mask per element.
#ifndef SOCP_GLOAD_BATCH
#define SOCP_GLOAD_BATCH 16
#endif
    constexpr int GT = NP * NQ, GB = SOCP_GLOAD_BATCH;
    // (the base made wave-uniform explicitly: a divergent-looking descriptor
    // would be waterfall-looped around every load)
    const uint64_t gpu = (uint64_t)Gp;
    const uint64_t gbase = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(gpu >> 32)) << 32) |
                           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)gpu);
    const __amdgpu_buffer_rsrc_t grs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)gbase, (short)0, __builtin_amdgcn_readfirstlane(k * n * (int)sizeof(double)), 0x00020000);
    int colk[NQ];  // byte offset of the lane's column in each column tile, or "out of range"
#pragma unroll
    for (int q = 0; q < NQ; ++q) colk[q] = 16 * q + cl < n ? (16 * q + cl) * k * 8 : 0x40000000;
#pragma unroll
    for (int b0 = 0; b0 < GT; b0 += GB) {
      uint64_t tmp[GB];
#pragma unroll
      for (int t = 0; t < GB; ++t) {
        const int e = b0 + t;
        if (e < GT) {
          const int pp = e / NQ, q = e % NQ;
          const int row = 4 * pp + g;
          const int off = row < k ? colk[q] + row * 8 : 0x40000000;
          tmp[t] = __builtin_bit_cast(uint64_t, __builtin_amdgcn_raw_buffer_load_b64(grs, off, 0, 0));
        }
      }
#pragma unroll
      for (int t = 0; t < GB; ++t) {
        const int e = b0 + t;
        if (e < GT) a_put(G[e / NQ][e % NQ], __longlong_as_double((long long)tmp[t]));
      }
    }
    }
    for (int e = lane; e < NKV * SH::KS; e += 64) LDS(O_KV + e) = 0.0;
    for (int e = lane; e < O_U + SH::UAL - O_A; e += 64) LDS(O_A + e) = 0.0;
    SYNC();
    if (lane < n) LDS(C_ + lane) = cv;
    if (lane < m) LDS(B_ + lane) = bv;
    if (lane < k) LDS(H_ + lane) = hv0;
    if (lane + 64 < k) LDS(H_ + 64 + lane) = hv1;
    for (int e0 = 0; e0 < mn; e0 += 64 * AB) {
#pragma unroll
      for (int t = 0; t < AB; ++t) {
        const int e = e0 + 64 * t + lane;
        if (e < mn) LDS(O_A + (e % m) * LDA + e / m) = av[t];
      }
      const int e1 = e0 + 64 * AB;
      if (e1 < mn) {
#pragma unroll
        for (int t = 0; t < AB; ++t) av[t] = (e1 + 64 * t + lane < mn) ? Ap[e1 + 64 * t + lane] : 0.0;
      }
    }
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
      LDS(IL + i) = e;  // 1/lambda_i of the POC elements (lambda = e)
    }
    for (int e = lane; e < NCS * NPAD; e += 64) LDS(O_U + e) = 0.0;
    if (lane < nc) {  // W = I, lambda = e: mu = wbar_0 = lambda_0 = 1, wbar_1 = lambda_1 = 0
      const int c = lane;
      LDS(cc(CC_MU, c)) = 1.0;
      LDS(cc(CC_IMU, c)) = 1.0;
      LDS(cc(CC_WB0, c)) = 1.0;
      LDS(cc(CC_I1, c)) = 0.5;
      LDS(cc(CC_W2, c)) = 0.0;
      LDS(cc(CC_L0, c)) = 1.0;
      LDS(cc(CC_AA, c)) = 1.0;
      LDS(cc(CC_IAA, c)) = 1.0;
      LDS(cc(CC_IL0, c)) = 1.0;
      LDS(cc(CC_IL0AA, c)) = 1.0;
      LDS(cc(CC_SA, c)) = 1.0;
      LDS(cc(CC_SAL, c)) = 0.5;
      LDS(cc(CC_WL, c)) = 0.0;
    }
    SYNC();
  }

  // ------------------------------------------------------ cone vector ops
  // The k-vector lives in two 64-element slots (element i = 64 s + lane).  Every
  // SOC operation of the reference (scale!/iscale!, iprod!/vprod!, the SOC
  // branch of compute_scaling, scmax) needs one or two per-cone dot products;
  // they come from cone_reduce, and each op below is straight-line code over
  // registers: the values a cone head holds (x_0, the cone constants) are
  // recomputed or read by every lane of the cone instead of being broadcast.

  // Per-cone (segmented) reduction of NV values per slot.  v[s][q] holds the
  // lane's contribution for element 64 s + lane; on return every lane of a cone
  // holds the cone total -- a sum, or a max for the values flagged in MX.  DPP
  // inclusive scan inside each slot, then the segment-end lanes hand their
  // partials over through LDS (a cone may span both slots).
  // The slots' scans run interleaved step by step (independent DPP chains
  // hide each other's latency); the DPP moves write every lane, so no old value
  // is materialised (lanes a pattern leaves unwritten fail the step's
  // predicate); all partials are read before any is used.
  template <int NV, unsigned MX>
  __device__ __forceinline__ void cone_reduce(double (&v)[2][NV]) {
    MARK_BEGIN("cone_reduce");
    LANE_IDS();
    constexpr int NS = KP > 64 ? 2 : 1;  // slots that can hold elements of this shape
    if (a.al_rows) {  // row-aligned cones: registers only
      const int R = a.al_rows;
      constexpr unsigned MXM = NS == 2 ? (MX | (MX << NV)) : MX;
      double w[NS * NV];
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int q = 0; q < NV; ++q) w[s * NV + q] = v[s][q];
      cone_allreduce_rows_n<NS * NV, MXM>(w, R);
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int q = 0; q < NV; ++q) v[s][q] = w[s * NV + q];
      return;
    }
    const int rl = lane & 15;
#define SOCP_SCAN_STEP(CTRL, OK)                                         \
  _Pragma("unroll") for (int s = 0; s < NS; ++s) {                       \
    const int st = ssl[s];                                               \
    const bool ok_ = (OK);                                               \
    _Pragma("unroll") for (int q = 0; q < NV; ++q) {                     \
      const double y = dpp_all<CTRL>(v[s][q]);                           \
      const double r = ((MX >> q) & 1) ? fmax(v[s][q], y) : v[s][q] + y; \
      v[s][q] = ok_ ? r : v[s][q];                                       \
    }                                                                    \
  }
    SOCP_SCAN_STEP(0x111, rl >= 1 && lane - 1 >= st)
    SOCP_SCAN_STEP(0x112, rl >= 2 && lane - 2 >= st)
    SOCP_SCAN_STEP(0x114, rl >= 4 && lane - 4 >= st)
    SOCP_SCAN_STEP(0x118, rl >= 8 && lane - 8 >= st)
    SOCP_SCAN_STEP(0x142, ((lane >> 4) & 1) && ((lane & ~15) - 1 >= st))
    SOCP_SCAN_STEP(0x143, lane >= 32 && 31 >= st)
#undef SOCP_SCAN_STEP
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (lane == sle[s]) {
#pragma unroll
        for (int q = 0; q < NV; ++q) LDS(O_PART + (q * NCS + ci[s]) * 2 + s) = v[s][q];
      }
    }
    SYNC();
    double pp[NS][NV][2];
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        pp[s][q][0] = LDS(O_PART + (q * NCS + ci[s]) * 2);
        pp[s][q][1] = LDS(O_PART + (q * NCS + ci[s]) * 2 + 1);
      }
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int q = 0; q < NV; ++q) {
        const double p0 = pp[s][q][0], p1 = pp[s][q][1];
        const double both = ((MX >> q) & 1) ? fmax(p0, p1) : p0 + p1;
        v[s][q] = spn[s] ? both : (s == 0 ? p0 : p1);
      }
  }

  // The scan half of cone_reduce for sums: the segment-end lanes leave the
  // two slot partials of every cone in O_PART; cone_tot(q, c) adds them (the
  // unused (cone, slot) entries stay zero).  For per-cone work done once per
  // cone (on "cone lanes", lane c < nc) instead of once per element.
  template <int NV>
  __device__ __forceinline__ void cone_partials(double (&v)[2][NV]) {
    MARK_BEGIN("cone_partials");
    LANE_IDS();
    constexpr int NS = KP > 64 ? 2 : 1;
    const int rl = lane & 15;
    if (a.al_rows) {  // row-aligned cones: every lane of the cone gets its total
      const int R = a.al_rows;
      double w[NS * NV];
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int q = 0; q < NV; ++q) w[s * NV + q] = v[s][q];
      cone_allreduce_rows_n<NS * NV, 0u>(w, R);
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int q = 0; q < NV; ++q) v[s][q] = w[s * NV + q];
    } else {
#define SOCP_SCAN_STEP(CTRL, OK)                         \
  _Pragma("unroll") for (int s = 0; s < NS; ++s) {       \
    const int st = ssl[s];                               \
    const bool ok_ = (OK);                               \
    _Pragma("unroll") for (int q = 0; q < NV; ++q) {     \
      const double y = dpp_all<CTRL>(v[s][q]);           \
      v[s][q] = ok_ ? v[s][q] + y : v[s][q];             \
    }                                                    \
  }
    SOCP_SCAN_STEP(0x111, rl >= 1 && lane - 1 >= st)
    SOCP_SCAN_STEP(0x112, rl >= 2 && lane - 2 >= st)
    SOCP_SCAN_STEP(0x114, rl >= 4 && lane - 4 >= st)
    SOCP_SCAN_STEP(0x118, rl >= 8 && lane - 8 >= st)
    SOCP_SCAN_STEP(0x142, ((lane >> 4) & 1) && ((lane & ~15) - 1 >= st))
    SOCP_SCAN_STEP(0x143, lane >= 32 && 31 >= st)
#undef SOCP_SCAN_STEP
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      if (lane == sle[s]) {
#pragma unroll
        for (int q = 0; q < NV; ++q) LDS(O_PART + (q * NCS + ci[s]) * 2 + s) = v[s][q];
      }
    }
    SYNC();
  }
  __device__ __forceinline__ double cone_tot(int q, int c) const {
    return LDS(O_PART + (q * NCS + c) * 2) + LDS(O_PART + (q * NCS + c) * 2 + 1);
  }

  __device__ __forceinline__ double ccv(int q, int c) const { return LDS(cc(q, c)); }

  // max over cones of the value the first lane of every cone stored at O_TOTC + off
  __device__ __forceinline__ double cone_max(int off) const {
    double t = -INFINITY, v[NCS];  // all reads in one round trip (the entries c >= nc are not used)
#pragma unroll
    for (int c = 0; c < NCS; ++c) v[c] = LDS(O_TOTC + off + c);
#pragma unroll
    for (int c = 0; c < NCS; ++c) t = c < nc ? fmax(t, v[c]) : t;
    return t;
  }

  // reciprocal and reciprocal square root: hardware estimate + Newton steps
  // (within an ulp or two of the IEEE quotient: the parity gates are relative
  // 1e-9, and these replace IEEE divisions in per-element and per-cone math)
  __device__ __forceinline__ static double rcp_nr(double d) { return recip(d); }

  // compute_scaling (scalings.jl:22-110) and ds = lam o lam (solver.jl:120).
  // Writes WB (wbar / sqrt(s/z)), LAM, IL (1/lambda of the POC elements), the
  // X = W^-1 G row coefficients CA, CBV, DS (write_ds: the iteration's
  // lam o lam; the KKT entry keeps its ds) and the per-cone constants; ll =
  // lam'lam.  Returns the DomainError flag; dm_aa flags a negative
  // lambda_0^2 - |lambda_1|^2 (scmax's sqrt, mats.jl:66), which the reference
  // raises later, at compute_step.
  // Two segmented reductions; the SOC cone math (norms, gamma, mu, lambda_0 and
  // the coefficients of the tail rows) runs once per cone on lane c, not once
  // per element.
  __device__ __forceinline__ bool scaling_op(double& ll, bool& dm_aa, bool write_ds) {
    MARK_BEGIN("scaling_op");
    if (SOCP_KO & 4096) {
      ll = 1.0;
      dm_aa = false;
      return false;
    }
    LANE_IDS();
    double v[2][3], zi[2], si[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = 64 * s + lane;
      zi[s] = LDS(Z_ + i);
      si[s] = LDS(S_ + i);
      const bool tail = kd[s] == 2;
      v[s][0] = tail ? zi[s] * zi[s] : 0.0;
      v[s][1] = tail ? si[s] * si[s] : 0.0;
      v[s][2] = tail ? zi[s] * si[s] : 0.0;
    }
    cone_partials<3>(v);
    MARK_BEGIN("scal_cone1");
    bool dm = false;
    // ---- cone lanes: the SOC branch of compute_scaling (scalings.jl:32-99)
    if (HOIST_CST ? lc_soc : (lane < nc && (int)LDS(O_CKIND + lane) == SOC_K)) {
      const int c = lane, o = HOIST_CST ? lc_off : (int)LDS(O_COFF + c);
      const double z0 = LDS(Z_ + o), s0 = LDS(S_ + o);
      const double onrmz = z0 * z0 - cone_tot(0, c), onrms = s0 * s0 - cone_tot(1, c);
      // the square roots and their reciprocals from one Newton-refined rsq each
      const double fz = rsqrt_nr(onrmz), fs = rsqrt_nr(onrms);
      const double nrmz = onrmz * fz, nrms = onrms * fs;
      const double zb0 = z0 * fz, sb0 = s0 * fs;
      const double nsum = zb0 * sb0 + cone_tot(2, c) * fz * fs;
      const double garg = (1.0 + nsum) * 0.5;
      const double rg = rsqrt_nr(garg);
      const double gamma = garg * rg;
      const double fg = 0.5 * rg;
      const double wb0 = (sb0 + zb0) * fg;
      const double ratio = nrms * fz, prod = nrms * nrmz;
      const double im = rsqrt_nr(ratio), mu = ratio * im, tmv1 = sqrt_nr(prod);
      const double mult = tmv1 * recip(zb0 + sb0 + 2.0 * gamma);
      const double l0 = gamma * tmv1;
      dm = (onrmz < 0.0) || (onrms < 0.0) || (garg < 0.0) || (ratio < 0.0) || (prod < 0.0);
      LDS(cc(CC_MU, c)) = mu;
      LDS(cc(CC_IMU, c)) = im;
      LDS(cc(CC_WB0, c)) = wb0;
      LDS(cc(CC_I1, c)) = recip(1.0 + wb0);
      LDS(cc(CC_L0, c)) = l0;
      LDS(cc(CC_AS, c)) = fs * fg;  // wbar_i = (s_i/|s| - z_i/|z|) / (2 gamma)
      LDS(cc(CC_AZ, c)) = fz * fg;
      LDS(cc(CC_BS, c)) = fs * (gamma + zb0) * mult;  // lambda_i (scalings.jl:91-97)
      LDS(cc(CC_BZ, c)) = fz * (gamma + sb0) * mult;
      LDS(WB + o) = wb0;
      LDS(LAM + o) = l0;
      LDS(CA + o) = -im;
      LDS(CBV + o) = -(1.0 + wb0) * im;
    }
    SYNC();
    MARK_BEGIN("scal_elem");
    // ---- elements: POC (scalings.jl:22-30) and the SOC tails
    double li[2], wbi[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = 64 * s + lane, c = ci[s];
      const bool poc = kd[s] == 0, tail = kd[s] == 2;
      // POC: one 1/sqrt(s z) gives sqrt(s/z) = s q, sqrt(z/s) = z q, sqrt(s z) = (s z) q
      const double pr = si[s] * zi[s];
      const double q = rsqrt_nr(pr);
      const double as = ccv(CC_AS, c), az = ccv(CC_AZ, c), bs = ccv(CC_BS, c), bz = ccv(CC_BZ, c);
      const double imu = ccv(CC_IMU, c), l0 = ccv(CC_L0, c);
      const double wt = si[s] * as - zi[s] * az;
      const double lt = si[s] * bs + zi[s] * bz;
      dm = dm || (poc && pr < 0.0);
      wbi[s] = poc ? zmul(si[s], q) : (tail ? wt : ccv(CC_WB0, c));
      li[s] = poc ? zmul(pr, q) : (tail ? lt : l0);
      if (poc || tail) {
        LDS(WB + i) = wbi[s];
        LDS(LAM + i) = li[s];
        LDS(CA + i) = poc ? zmul(zi[s], q) : imu;
        LDS(CBV + i) = poc ? 0.0 : wt * imu;
        if (poc) LDS(IL + i) = q;
        if (write_ds) LDS(DS + i) = -(poc ? li[s] * li[s] : (l0 * li[s] + l0 * li[s]));  // -ds: the RHS
      }
      // lam o lam head (vprod!, vectors.jl:58-75) and |lambda_1|^2 (POC: the
      // cone's sum of lambda_i^2, its share of lam'lam), |wbar_1|^2, wbar_1'lambda_1
      v[s][0] = (poc || tail) ? li[s] * li[s] : 0.0;
      v[s][1] = tail ? wbi[s] * wbi[s] : 0.0;
      v[s][2] = tail ? wbi[s] * li[s] : 0.0;
    }
    cone_partials<3>(v);
    MARK_BEGIN("scal_cone2");
    bool da = false;
    double tl = 0.0;
    if (lane < nc) {
      const int c = lane;
      const double l1 = cone_tot(0, c);
      if (HOIST_CST ? lc_soc : (int)LDS(O_CKIND + c) == SOC_K) {
        const int o = HOIST_CST ? lc_off : (int)LDS(O_COFF + c);
        const double l0 = LDS(cc(CC_L0, c));
        const double aa = l0 * l0 - l1;
        da = aa < 0.0;
        const double sa = rsqrt_nr(aa);
        LDS(cc(CC_W2, c)) = cone_tot(1, c);
        LDS(cc(CC_WL, c)) = cone_tot(2, c);
        LDS(cc(CC_AA, c)) = aa;
        LDS(cc(CC_IAA, c)) = recip(aa);
        LDS(cc(CC_IL0, c)) = recip(l0);
        LDS(cc(CC_IL0AA, c)) = recip(l0 * aa);
        LDS(cc(CC_SA, c)) = sa;
        LDS(cc(CC_SAL, c)) = recip(sa * l0 + 1.0);
        tl = l0 * l0 + l1;
        if (write_ds) LDS(DS + o) = -tl;
      } else {
        tl = l1;
      }
    }
    SYNC();
    ll = wsum(tl);
    dm_aa = __any(da);
    return __any(dm);
  }

#ifndef SOCP_RESID_SCAL
#define SOCP_RESID_SCAL 1  // MP_ITER: residuals and compute_scaling interleaved (0: back to back)
#endif
  // The per-cone SOC branch of compute_scaling (scalings.jl:32-99) on cone lane
  // c = lane, computed on every lane (branch-free: its instructions share the
  // caller's scheduling region) and stored by the SOC cone lanes only.
  struct ScalCone1 {
    double mu, im, wb0, i1, l0, as, az, bs, bz;
    bool dm;
  };
  __device__ __forceinline__ ScalCone1 scal_cone1_math(int o, int c) const {
    ScalCone1 r;
    const double z0 = LDS(Z_ + o), s0 = LDS(S_ + o);
    const double onrmz = z0 * z0 - cone_tot(0, c), onrms = s0 * s0 - cone_tot(1, c);
    const double fz = rsqrt_nr(onrmz), fs = rsqrt_nr(onrms);
    const double nrmz = onrmz * fz, nrms = onrms * fs;
    const double zb0 = z0 * fz, sb0 = s0 * fs;
    const double nsum = zb0 * sb0 + cone_tot(2, c) * fz * fs;
    const double garg = (1.0 + nsum) * 0.5;
    const double rg = rsqrt_nr(garg);
    const double gamma = garg * rg;
    const double fg = 0.5 * rg;
    r.wb0 = (sb0 + zb0) * fg;
    const double ratio = nrms * fz, prod = nrms * nrmz;
    r.im = rsqrt_nr(ratio);
    r.mu = ratio * r.im;
    const double tmv1 = sqrt_nr(prod);
    const double mult = tmv1 * recip(zb0 + sb0 + 2.0 * gamma);
    r.l0 = gamma * tmv1;
    r.dm = (onrmz < 0.0) || (onrms < 0.0) || (garg < 0.0) || (ratio < 0.0) || (prod < 0.0);
    r.i1 = recip(1.0 + r.wb0);
    r.as = fs * fg;
    r.az = fz * fg;
    r.bs = fs * (gamma + zb0) * mult;
    r.bz = fz * (gamma + sb0) * mult;
    return r;
  }
  __device__ __forceinline__ void scal_cone1_store(const ScalCone1& r, int o, int c) {
    LDS(cc(CC_MU, c)) = r.mu;
    LDS(cc(CC_IMU, c)) = r.im;
    LDS(cc(CC_WB0, c)) = r.wb0;
    LDS(cc(CC_I1, c)) = r.i1;
    LDS(cc(CC_L0, c)) = r.l0;
    LDS(cc(CC_AS, c)) = r.as;  // wbar_i = (s_i/|s| - z_i/|z|) / (2 gamma)
    LDS(cc(CC_AZ, c)) = r.az;
    LDS(cc(CC_BS, c)) = r.bs;  // lambda_i (scalings.jl:91-97)
    LDS(cc(CC_BZ, c)) = r.bz;
    LDS(WB + o) = r.wb0;
    LDS(LAM + o) = r.l0;
    LDS(CA + o) = -r.im;
    LDS(CBV + o) = -(1.0 + r.wb0) * r.im;
  }

  // gemv_Gt hook: the cone-lane chain in the first batch of G'z
  struct ScalHook {
    Small& S;
    ScalCone1& r;
    int o, c;
    template <int B>
    __device__ __forceinline__ void run() {
      if constexpr (B == 0) r = S.scal_cone1_math(o, c);
    }
  };

  // MP_ITER: the residuals (solver.jl:109-118) and compute_scaling (:106) with
  // ds = lam o lam (:120) in one pass.  They are independent (the scaling
  // reads z and s, the residuals x, y, z, s), so their phases share
  // scheduling regions: the scaling's cone-lane chains (rsqrt / recip
  // latency on three lanes) run inside the residuals' G'z pass and beside
  // their G x pass (VALU issue), the element part beside the A products (LDS
  // latency).  The same operations as residuals() then scaling_op(): the
  // results are bitwise the same.  Returns the DomainError flag.
  __device__ __forceinline__ bool resid_scaling(double& nd, double& np_, double& gap, double& ll, bool& dm_aa) {
    MARK_BEGIN("resid_scaling");
    LANE_IDS();
    constexpr int NS = KP > 64 ? 2 : 1;
    double cq[NQ], xq[NQ], zv[NS], sv[NS];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      cq[q] = LDS(C_ + 16 * q + cl);
      xq[q] = LDS(X_ + 16 * q + cl);
    }
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      zv[t] = LDS(Z_ + 64 * t + lane);
      sv[t] = LDS(S_ + 64 * t + lane);
    }
    // ---- scaling, first reduction: |z_1|^2, |s_1|^2, z_1's_1 per cone
    double v[2][3], zi[2], si[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = 64 * s + lane;
      zi[s] = LDS(Z_ + i);
      si[s] = LDS(S_ + i);
      const bool tail = kd[s] == 2;
      v[s][0] = tail ? zi[s] * zi[s] : 0.0;
      v[s][1] = tail ? si[s] * si[s] : 0.0;
      v[s][2] = tail ? zi[s] * si[s] : 0.0;
    }
    cone_partials<3>(v);
    // ---- the cone-lane chain inside G'z's first batch
    const bool socl = HOIST_CST ? lc_soc : (lane < nc && (int)LDS(O_CKIND + lane) == SOC_K);
    const int cc_ = lane < nc ? lane : 0;
    const int oc = socl ? (HOIST_CST ? lc_off : (int)LDS(O_COFF + lane)) : 0;
    ScalCone1 c1;
    double acc[NQ], at[NQ];
    gemv_Gt(Z_, acc, ScalHook{*this, c1, oc, cc_});
    if (socl) scal_cone1_store(c1, oc, cc_);
    bool dm = socl && c1.dm;
    SYNC();
    // ---- the elements (POC, scalings.jl:22-30; SOC tails) beside A'y
    MARK_BEGIN("scal_elem");
    double li[2], wbi[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = 64 * s + lane, c = ci[s];
      const bool poc = kd[s] == 0, tail = kd[s] == 2;
      const double pr = si[s] * zi[s];
      const double q = rsqrt_nr(pr);
      const double as = ccv(CC_AS, c), az = ccv(CC_AZ, c), bs = ccv(CC_BS, c), bz = ccv(CC_BZ, c);
      const double imu = ccv(CC_IMU, c), l0 = ccv(CC_L0, c);
      const double wt = si[s] * as - zi[s] * az;
      const double lt = si[s] * bs + zi[s] * bz;
      dm = dm || (poc && pr < 0.0);
      wbi[s] = poc ? zmul(si[s], q) : (tail ? wt : ccv(CC_WB0, c));
      li[s] = poc ? zmul(pr, q) : (tail ? lt : l0);
      if (poc || tail) {
        LDS(WB + i) = wbi[s];
        LDS(LAM + i) = li[s];
        LDS(CA + i) = poc ? zmul(zi[s], q) : imu;
        LDS(CBV + i) = poc ? 0.0 : wt * imu;
        if (poc) LDS(IL + i) = q;
        LDS(DS + i) = -(poc ? li[s] * li[s] : (l0 * li[s] + l0 * li[s]));  // -ds: the RHS
      }
      v[s][0] = (poc || tail) ? li[s] * li[s] : 0.0;
      v[s][1] = tail ? wbi[s] * wbi[s] : 0.0;
      v[s][2] = tail ? wbi[s] * li[s] : 0.0;
    }
    At_mv(Y_, at);
    cone_partials<3>(v);
    // ---- rd, the second cone-lane part beside A x and G x + s - h
    double d2 = 0.0, zs = 0.0;
    if (g == 0) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int j = 16 * q + cl;
        if (j < n) {
          const double vv = (at[q] + acc[q]) + cq[q];
          LDS(RD + j) = -vv;  // the residuals are stored negated: the affine RHS (solver.jl:124)
          d2 = fma(vv, vv, d2);
        }
      }
    }
    const double p2 = A_mv(X_, B_, RP, O_A, true);
    bool da = false;
    double tl = 0.0;
    {
      MARK_BEGIN("scal_cone2");
      const double l1 = cone_tot(0, cc_);
      const double l0 = LDS(cc(CC_L0, cc_));
      const double aa = l0 * l0 - l1;
      const double sa = rsqrt_nr(aa);
      const double w2 = cone_tot(1, cc_), wl = cone_tot(2, cc_);
      const double iaa = recip(aa), il0 = recip(l0), il0aa = recip(l0 * aa), sal = recip(sa * l0 + 1.0);
      gemv_G_r<true>(xq, S_, H_, DZ);
      if (lane < nc) {
        if (socl) {
          da = aa < 0.0;
          LDS(cc(CC_W2, cc_)) = w2;
          LDS(cc(CC_WL, cc_)) = wl;
          LDS(cc(CC_AA, cc_)) = aa;
          LDS(cc(CC_IAA, cc_)) = iaa;
          LDS(cc(CC_IL0, cc_)) = il0;
          LDS(cc(CC_IL0AA, cc_)) = il0aa;
          LDS(cc(CC_SA, cc_)) = sa;
          LDS(cc(CC_SAL, cc_)) = sal;
          tl = l0 * l0 + l1;
          LDS(DS + oc) = -tl;
        } else {
          tl = l1;
        }
      }
    }
    SYNC();
#pragma unroll
    for (int t = 0; t < NS; ++t)
      if (64 * t + lane < k) zs += zv[t] * sv[t];
    double r3[3] = {d2, p2, zs};  // the three whole-wave sums in one interleaved scan
    dpp_scan<3>(r3, lane, 0, false);
    nd = sqrt(readlane_d(r3[0], 63));
    np_ = sqrt(readlane_d(r3[1], 63));
    gap = readlane_d(r3[2], 63);
    ll = wsum(tl);
    dm_aa = __any(da);
    return __any(dm);
  }

  // First half of solve_kkt(::DenseSolver) (densesolver.jl:61-66):
  //   k0 = lam^-1 o ds (iprod!), k1 = W k0 (scale!), k2 = dz - k1,
  //   t2 = iWiW k2 = W^-1 (W^-1 k2).
  // Every SOC dot product the chain needs follows by linearity from three dots
  // of the inputs, taken in ONE reduction: t = lambda_1'ds_1 (iprod!'s),
  // u = wbar_1'ds_1, w = wbar_1'dz_1, with the scaling's wbar_1'lambda_1 and
  // |wbar_1|^2:  wbar_1'k0_1 = -ds_0 WL/aa + u/lambda_0 + WL t/(lambda_0 aa),
  // wbar_1'k1_1 = mu (delta + (k0_0 + delta/(1+wbar_0)) |wbar_1|^2), and the
  // second W^-1 reuses the first one's dot.  POC: k0 = ds / lambda by the
  // reciprocal kept in IL.  In: DS, DZ.  Out: K0, K2, T2, DLT (per cone).
  __device__ __forceinline__ void solve_head() {
    MARK_BEGIN("solve_head");
    if (SOCP_KO & 8192) return;
    LANE_IDS();
    double v[2][3], x[2], x0[2], dz[2], dz0[2], lam[2], wb[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = 64 * s + lane;
      x[s] = LDS(DS + i);
      x0[s] = LDS(DS + eo[s]);
      dz[s] = LDS(DZ + i);
      dz0[s] = LDS(DZ + eo[s]);
      lam[s] = LDS(LAM + i);
      wb[s] = LDS(WB + i);
      const bool tail = kd[s] == 2;
      v[s][0] = tail ? lam[s] * x[s] : 0.0;
      v[s][1] = tail ? wb[s] * x[s] : 0.0;
      v[s][2] = tail ? wb[s] * dz[s] : 0.0;
    }
    // the scaling's per-cone constants and the element coefficients are read
    // before the reduction: their LDS latency hides under its DPP chain
    double cst[2][12];
    auto read_cst = [&]() {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = 64 * s + lane, c = ci[s];
      cst[s][0] = ccv(CC_L0, c);
      cst[s][1] = ccv(CC_IAA, c);
      cst[s][2] = ccv(CC_IL0, c);
      cst[s][3] = ccv(CC_IL0AA, c);
      cst[s][4] = ccv(CC_MU, c);
      cst[s][5] = ccv(CC_IMU, c);
      cst[s][6] = ccv(CC_WB0, c);
      cst[s][7] = ccv(CC_I1, c);
      cst[s][8] = ccv(CC_W2, c);
      cst[s][9] = ccv(CC_WL, c);
      cst[s][10] = LDS(IL + i);
      cst[s][11] = LDS(CA + i);
    }
    };
    if constexpr (HOIST_CST) read_cst();
    cone_reduce<3, 0>(v);
    STAMP_X(8);
    MARK_BEGIN("head_post");
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = 64 * s + lane, c = ci[s];
      const double t = v[s][0], u = v[s][1], w = v[s][2];
#define CST(j, expr) (HOIST_CST ? cst[s][j] : (expr))
      const double l0 = CST(0, ccv(CC_L0, c)), iaa = CST(1, ccv(CC_IAA, c)), il0 = CST(2, ccv(CC_IL0, c)),
                   il0aa = CST(3, ccv(CC_IL0AA, c));
      const double mu = CST(4, ccv(CC_MU, c)), imu = CST(5, ccv(CC_IMU, c)), wb0 = CST(6, ccv(CC_WB0, c)),
                   i1 = CST(7, ccv(CC_I1, c));
      const double w2 = CST(8, ccv(CC_W2, c)), wl = CST(9, ccv(CC_WL, c));
      // iprod! (vectors.jl:105-125)
      const double k00 = (x0[s] * l0 - t) * iaa;
      const double k0t = -(x0[s] * lam[s] * iaa) + x[s] * il0 + lam[s] * t * il0aa;
      const double dlt = -(x0[s] * wl * iaa) + u * il0 + wl * t * il0aa;  // wbar_1'k0_1
      // scale! (scalings.jl:159-165)
      const double k10 = mu * (wb0 * k00 + dlt);
      const double k1t = mu * (k0t + (k00 + dlt * i1) * wb[s]);
      const double k20 = dz0[s] - k10;
      const double a1 = w - mu * (dlt + (k00 + dlt * i1) * w2);  // wbar_1'k2_1
      // iscale! twice (scalings.jl:167-173)
      const double cy = a1 * i1 - k20;
      const double y0 = imu * (wb0 * k20 - a1);
      const double a2 = imu * (a1 + cy * w2);
      // POC: elementwise, with 1/lambda and 1/w = CA
      const double k0p = x[s] * CST(10, LDS(IL + i));
      const double k2p = dz[s] - wb[s] * k0p;
      const double ca = CST(11, LDS(CA + i));
      const bool poc = kd[s] == 0, hd = kd[s] == 1;
      const double k0 = poc ? k0p : (hd ? k00 : k0t);
      const double k2 = poc ? k2p : dz[s] - (hd ? k10 : k1t);
      const double yt = imu * (k2 + cy * wb[s]);
      const double zs = hd ? imu * (wb0 * y0 - a2) : imu * (yt + (a2 * i1 - y0) * wb[s]);
      if (kd[s] != 3) {
        LDS(K0 + i) = k0;
        LDS(K2 + i) = k2;
        LDS(T2 + i) = poc ? ca * (ca * k2p) : zs;
      }
      if (hd) LDS(cc(CC_DLT, c)) = dlt;
    }
    SYNC();
  }

  // Second half of solve_kkt (densesolver.jl:83-88): cz = iWiW k1 = W^-1 (W^-1 k1),
  // k0 -= W cz (W cz = W^-1 k1 = y), cs = W k0.  wbar_1'(k0 - y)_1 is DLT
  // (solve_head's) minus wbar_1'y_1, so cs needs no reduction of its own.
  // With do_step, compute_step (mats.jl:30-40) of the direction
  // (solver.jl:128-130, 143-145) follows: kt3 = W rz and kt2 = W^-1 rs are y
  // and k0 - y exactly; and the dot kt2'kt3 (rho's, solver.jl:132) and each
  // cone's kt2'kt3 (the head of kt2 o kt3, :136) come out of the step's
  // reduction.  In: K1 (= G cx - k2), K0.  Out: RZ, RS, and with do_step
  // T1 = kt3, K0 = kt2, KK (per cone), O_TOTC[1][0] = kt2'kt3, the step
  // length (dom: DomainError).
  __device__ __forceinline__ double solve_tail(bool do_step, bool dm_aa, int& dom) {
    MARK_BEGIN("solve_tail");
    if (SOCP_KO & 16384) {
      dom = 0;
      return 1.0;
    }
    LANE_IDS();
    double v[2][3], k1[2], k10[2], k0[2], k00[2], wb[2], lam[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = 64 * s + lane;
      k1[s] = LDS(K1 + i);
      k10[s] = LDS(K1 + eo[s]);
      k0[s] = LDS(K0 + i);
      k00[s] = LDS(K0 + eo[s]);
      wb[s] = LDS(WB + i);
      lam[s] = LDS(LAM + i);
      const bool tail = kd[s] == 2;
      v[s][0] = tail ? wb[s] * k1[s] : 0.0;
      v[s][1] = tail ? lam[s] * k1[s] : 0.0;
      v[s][2] = tail ? lam[s] * k0[s] : 0.0;
    }
    double cst[2][12];  // read before the reduction (as in solve_head)
    auto read_cst = [&]() {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = 64 * s + lane, c = ci[s];
      cst[s][0] = ccv(CC_MU, c);
      cst[s][1] = ccv(CC_IMU, c);
      cst[s][2] = ccv(CC_WB0, c);
      cst[s][3] = ccv(CC_I1, c);
      cst[s][4] = ccv(CC_W2, c);
      cst[s][5] = ccv(CC_WL, c);
      cst[s][6] = LDS(CA + i);
      cst[s][7] = ccv(CC_DLT, c);
      cst[s][8] = ccv(CC_SA, c);
      cst[s][9] = ccv(CC_L0, c);
      cst[s][10] = ccv(CC_SAL, c);
      cst[s][11] = LDS(IL + i);
    }
    };
    if constexpr (HOIST_CST) read_cst();
    cone_reduce<3, 0>(v);
    STAMP_X(9);
    MARK_BEGIN("tail_post1");
    double y[2], y0v[2], kn[2], kn0[2], ly[2], lkn[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = 64 * s + lane, c = ci[s];
      const double a1 = v[s][0];
      const double mu = CST(0, ccv(CC_MU, c)), imu = CST(1, ccv(CC_IMU, c)), wb0 = CST(2, ccv(CC_WB0, c)),
                   i1 = CST(3, ccv(CC_I1, c));
      const double w2 = CST(4, ccv(CC_W2, c)), wl = CST(5, ccv(CC_WL, c));
      const double ca = CST(6, LDS(CA + i));
      const bool poc = kd[s] == 0, hd = kd[s] == 1;
      const double cy = a1 * i1 - k10[s];
      const double y0 = imu * (wb0 * k10[s] - a1);
      const double a2 = imu * (a1 + cy * w2);  // wbar_1'y_1
      y[s] = poc ? ca * k1[s] : (hd ? y0 : imu * (k1[s] + cy * wb[s]));
      const double zs = hd ? imu * (wb0 * y0 - a2) : imu * (y[s] + (a2 * i1 - y0) * wb[s]);
      y0v[s] = y0;
      kn[s] = k0[s] - y[s];
      kn0[s] = k00[s] - y0;
      const double del = CST(7, ccv(CC_DLT, c)) - a2;  // wbar_1'kn_1
      const double cs = poc ? wb[s] * kn[s]
                            : (hd ? mu * (wb0 * kn0[s] + del) : mu * (kn[s] + (kn0[s] + del * i1) * wb[s]));
      ly[s] = imu * (v[s][1] + cy * wl);  // lambda_1'y_1
      lkn[s] = v[s][2] - ly[s];           // lambda_1'kn_1
      if (kd[s] != 3) {
        LDS(RZ + i) = poc ? ca * y[s] : zs;
        LDS(RS + i) = cs;
      }
    }
    if (!do_step) {
      SYNC();
      return 0.0;
    }
    // scmax (mats.jl:42-86) of kt3 = y and kt2 = kn, and kt2'kt3
    double w[2][5], r1y[2], r1k[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = 64 * s + lane, c = ci[s];
      if (kd[s] != 3) {
        LDS(T1 + i) = y[s];
        LDS(K0 + i) = kn[s];
      }
      const bool tail = kd[s] == 2, poc = kd[s] == 0, real = kd[s] != 3;
      const double sa = CST(8, ccv(CC_SA, c)), l0 = CST(9, ccv(CC_L0, c)), sal = CST(10, ccv(CC_SAL, c));
      r1y[s] = sa * l0 * y0v[s] - sa * ly[s];
      r1k[s] = sa * l0 * kn0[s] - sa * lkn[s];
      const double cyy = (r1y[s] + y0v[s]) * sal, cyk = (r1k[s] + kn0[s]) * sal;
      const double qy = sa * (y[s] - cyy * sa * lam[s]), qk = sa * (kn[s] - cyk * sa * lam[s]);
      const double il = CST(11, LDS(IL + i));
      w[s][0] = tail ? qy * qy : 0.0;
      w[s][1] = tail ? qk * qk : 0.0;
      w[s][2] = poc ? -y[s] * il : -INFINITY;
      w[s][3] = poc ? -kn[s] * il : -INFINITY;
      w[s][4] = real ? y[s] * kn[s] : 0.0;
    }
    cone_reduce<5, 0xC>(w);
    STAMP_X(10);
    MARK_BEGIN("tail_post2");
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int c = ci[s];
      if (64 * s >= k || kd[s] == 3 || 64 * s + lane != eo[s]) continue;
      const double sa = CST(8, ccv(CC_SA, c));
#undef CST
      const double vy = sqrt_nr(w[s][0]) - sa * r1y[s];
      const double vk = sqrt_nr(w[s][1]) - sa * r1k[s];
      LDS(O_TOTC + c) = kd[s] == 0 ? fmax(w[s][2], w[s][3]) : fmax(vy, vk);
      LDS(cc(CC_KK, c)) = w[s][4];
    }
    SYNC();
    dom = dm_aa ? 1 : 0;
    const double t = fmax(cone_max(0), 0.0);
    return !(t > 1.0) ? 1.0 : (t == INFINITY ? 0.0 : recip(t));  // min(1, 1/t)
  }

  // rho, sigma, mu (solver.jl:132-134) and the corrector right-hand side
  // (:136-140): kt1 = kt2 o kt3, ds += sigma mu e - kt1, dx, dy, dz *= 1 - sigma.
  // kt2'kt3 and the SOC heads of kt2 o kt3 come from solve_tail's reduction.
  // In: K0 (kt2), T1 (kt3), KK, DS, DZ, RD, RP.
  __device__ __forceinline__ void affine_post(double tstep, double ll) {
    MARK_BEGIN("affine_post");
    if (SOCP_KO & 32768) return;
    LANE_IDS();
    double kk = 0.0, kv[NCS];  // one round trip
#pragma unroll
    for (int c = 0; c < NCS; ++c) kv[c] = LDS(cc(CC_KK, c));
#pragma unroll
    for (int c = 0; c < NCS; ++c) kk = c < nc ? kk + kv[c] : kk;
    const double t = tstep;
    const double rho = 1.0 - t - t * t * kk / ll;
    const double cr = isnan(rho) ? rho : (rho < 0.0 ? 0.0 : (rho > 1.0 ? 1.0 : rho));
    const double sig = ipow(cr, a.sigma_exp);  // max(0,min(1,rho))^3 (solver.jl:133)
    const double mu_ipm = ll / a.deg;
    const double scf = 1.0 - sig;
    const double smu = sig * mu_ipm;
    if constexpr (HOIST_CST) {
      // every read first (one round trip; n, m <= 64 here), then the updates
      double a2[2], a3[2], a20[2], a30[2], kkc[2], dsv[2], dzv[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int i = 64 * s + lane;
        a2[s] = LDS(K0 + i);
        a3[s] = LDS(T1 + i);
        a20[s] = LDS(K0 + eo[s]);
        a30[s] = LDS(T1 + eo[s]);
        kkc[s] = LDS(cc(CC_KK, ci[s]));
        dsv[s] = LDS(DS + i);
        dzv[s] = LDS(DZ + i);
      }
      const double rdv = LDS(RD + lane), rpv = LDS(RP + (lane < MPAD ? lane : 0));
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int i = 64 * s + lane;
        if (kd[s] == 3) continue;
        const double kt1 = kd[s] == 0 ? a2[s] * a3[s] : (kd[s] == 1 ? kkc[s] : a20[s] * a3[s] + a30[s] * a2[s]);
        const double e = kd[s] == 2 ? 0.0 : 1.0;
        LDS(DS + i) = dsv[s] + (smu * e - kt1);
        LDS(DZ + i) = dzv[s] * scf;
      }
      if (lane < n) LDS(RD + lane) = rdv * scf;
      if (lane < m) LDS(RP + lane) = rpv * scf;
      SYNC();
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int i = 64 * s + lane;
        if (kd[s] == 3) continue;
        const double a2 = LDS(K0 + i), a3 = LDS(T1 + i);
        const double a20 = LDS(K0 + eo[s]), a30 = LDS(T1 + eo[s]);
        const double kt1 = kd[s] == 0 ? a2 * a3 : (kd[s] == 1 ? LDS(cc(CC_KK, ci[s])) : a20 * a3 + a30 * a2);
        const double e = kd[s] == 2 ? 0.0 : 1.0;
        LDS(DS + i) = LDS(DS + i) + (smu * e - kt1);
        LDS(DZ + i) = LDS(DZ + i) * scf;
      }
      for (int j = lane; j < n; j += 64) LDS(RD + j) = LDS(RD + j) * scf;
      for (int i = lane; i < m; i += 64) LDS(RP + i) = LDS(RP + i) * scf;
      SYNC();
    }
  }

  // max_step(-iz), max_step(iz) (mats.jl:1-28) for the initial shift (solver.jl:88-101)
  __device__ __forceinline__ void maxstep_op(int xv, double& alphp, double& alphd) {
    MARK_BEGIN("maxstep_op");
    LANE_IDS();
    double v[2][3], x[2], x0[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int i = 64 * s + lane;
      x[s] = LDS(xv + i);
      x0[s] = LDS(xv + eo[s]);
      v[s][0] = kd[s] == 2 ? x[s] * x[s] : 0.0;
      v[s][1] = kd[s] == 0 ? x[s] : -INFINITY;
      v[s][2] = kd[s] == 0 ? -x[s] : -INFINITY;
    }
    cone_reduce<3, 0x6>(v);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if (64 * s >= k || kd[s] == 3 || 64 * s + lane != eo[s]) continue;
      const double nr = sqrt_nr(v[s][0]);
      const bool poc = kd[s] == 0;
      LDS(O_TOTC + ci[s]) = poc ? v[s][1] : nr + x0[s];
      LDS(O_TOTC + NCS + ci[s]) = poc ? v[s][2] : nr - x0[s];
    }
    SYNC();
    alphp = cone_max(0);
    alphd = cone_max(NCS);
  }

  // U[c,:] = (sum_{i in cone c} w_i G[i,:]) / (1+wb0), w_head = -(1+wb0), w_tail = wb_i
  // The cone descriptors come from the kernel arguments (scalar loads); the
  // row steps a cone covers are taken four at a time, their four weight reads
  // issued together (one LDS round trip per four row steps), the weights
  // masked branch-free.
  __device__ __forceinline__ void compute_U() {
    MARK_BEGIN("compute_U");
    LANE_IDS();
    // HOIST_CST shapes: every row's weight read once, in one round trip
    double wall[HOIST_CST ? NP : 1];
    if constexpr (HOIST_CST) {
#pragma unroll
      for (int pp = 0; pp < NP; ++pp) wall[pp] = LDS(WB + 4 * pp + g);
    }
#if SOCP_U_LANECONES
    // every SOC cone's offset, dim, head weight and 1/(1+wb0) on its cone lane
    // (lane c < nc), read in one round trip with the row weights; the loop
    // takes them by readlane (no scalar-memory or LDS wait per cone)
    bool socl = false;
    int ol = 0, dl = 0;
    double hwl = 0.0, invl = 0.0;
    if (lane < nc) {
      socl = HOIST_CST ? lc_soc : (int)LDS(O_CKIND + lane) == SOC_K;
      ol = HOIST_CST ? lc_off : (int)LDS(O_COFF + lane);
      dl = HOIST_CST ? lc_dim : (int)LDS(O_CDIM + lane);
      hwl = -(1.0 + LDS(WB + ol));
      invl = LDS(cc(CC_I1, lane));
    }
    for (uint64_t mk = __ballot(socl); mk; mk &= mk - 1) {
      const int c = __builtin_ctzll(mk);
      const int o = __builtin_amdgcn_readlane(ol, c), d = __builtin_amdgcn_readlane(dl, c);
      const double hw = readlane_d(hwl, c);  // the head row's weight
      const double inv = readlane_d(invl, c);
#else
    for (int c = 0; c < nc; ++c) {
      if (a.cones.kind[c] != SOC_K) continue;
      const int o = a.cones.offs[c], d = a.cones.dim[c];
      const double hw = -(1.0 + LDS(WB + o));  // the head row's weight
      const double inv = LDS(cc(CC_I1, c));
#endif
      const int p0 = o >> 2, p1 = (o + d + 3) >> 2;  // row steps [p0, p1) meet the cone
      double acc[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) acc[q] = 0.0;
#pragma unroll
      for (int pb = 0; pb < NP; pb += 4) {
        if (pb + 4 <= p0 || pb >= p1) continue;  // wave-uniform
        constexpr int U4 = 4;
        double w[U4];
#pragma unroll
        for (int u = 0; u < U4; ++u) {
          const int row = 4 * (pb + u) + g;  // < KP: in the LDS k-vector
          if constexpr (HOIST_CST)
            w[u] = (pb + u < NP) ? wall[pb + u < NP ? pb + u : 0] : 0.0;
          else
            w[u] = (pb + u < NP) ? LDS(WB + row) : 0.0;
        }
#pragma unroll
        for (int u = 0; u < U4; ++u) {
          const int row = 4 * (pb + u) + g;
          const bool in = row >= o && row < o + d;
          const double wu = in ? (row == o ? hw : w[u]) : 0.0;
          if (pb + u < NP) {
            {
              double gr[NQ];
              a_get_row<NQ>(G[pb + u < NP ? pb + u : 0], gr);
#pragma unroll
              for (int q = 0; q < NQ; ++q) acc[q] = fma(wu, gr[q], acc[q]);
            }
          }
        }
      }
#pragma unroll
      for (int q = 0; q < NQ; ++q) acc[q] = rows_sum(acc[q]);
      if (g == 0) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) LDS(O_U + c * NPAD + 16 * q + cl) = acc[q] * inv;
      }
    }
    SYNC();
  }

  // ----------------------------------------------------- H = X'X (+A'A)
#ifndef SOCP_SYRK_PIPE
#define SOCP_SYRK_PIPE 2  // 2: row coefficients two steps ahead, U rows one step ahead
#endif
#ifndef SOCP_SYRK_M
#define SOCP_SYRK_M 1
#define SOCP_SYRK_L 2
#define SOCP_SYRK_V 8
#endif
  // row step pp of X = W^-1 G: X[i,:] = CA_i G[i,:] + CBV_i U[cone(i),:]
  __device__ __forceinline__ void genX(int pp, double (&X)[NQ]) {
    LANE_IDS();
    const int row = 4 * pp + g;
    const double cav = LDS(CA + row), cbv = LDS(CBV + row);
    const int cid = ((int)LDS(O_RC + row)) >> 2;
#pragma unroll
    for (int q = 0; q < NQ; ++q) X[q] = fma(cav, a_get(G[pp][q]), cbv * LDS(O_U + cid * NPAD + 16 * q + cl));
  }
  // genX in two halves, for a two-deep pipeline: the row coefficients (and the
  // cone id that addresses U) first, the U row and the products a step later
  struct XCoef {
    double ca, cb;
    int ub;  // LDS index of the cone's U row + cl
  };
  // (UBT shapes: the lane ids of form_H, computed once for the whole product,
  // and the U row from the launch's table)
  __device__ __forceinline__ XCoef genX_a(int pp, int g_, int cl_) {
    XCoef c;
    if constexpr (SH::UBT) {
      const int row = 4 * pp + g_;
      c.ca = LDS(CA + row);
      c.cb = LDS(CBV + row);
      c.ub = ubt(row) + cl_;  // O_U + cone(row) * NPAD
    } else {
      LANE_IDS();
      const int row = 4 * pp + g;
      c.ca = LDS(CA + row);
      c.cb = LDS(CBV + row);
      c.ub = O_U + (((int)LDS(O_RC + row)) >> 2) * NPAD + cl;
    }
    return c;
  }
  __device__ __forceinline__ void genX_b(int pp, const XCoef& c, double (&X)[NQ]) {
    double u[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) u[q] = LDS(c.ub + 16 * q);
    {
      double gr[NQ];
      a_get_row<NQ>(G[pp], gr);
#pragma unroll
      for (int q = 0; q < NQ; ++q) X[q] = fma(c.ca, gr[q], c.cb * u[q]);
    }
  }
  static constexpr bool diag_tile(int t) {
    for (int i = 0; i < NQ; ++i)
      if (tri(i, i) == t) return true;
    return false;
  }
  __device__ __forceinline__ void form_H(bool addAA) {
    MARK_BEGIN("form_H");
    LANE_IDS();
    if (SOCP_KO & 65536) {  // H = I
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) T[t][r] = (diag_tile(t) && g + 4 * r == cl) ? 1.0 : 0.0;
      return;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) T[t] = (d4){0.0, 0.0, 0.0, 0.0};
#if SOCP_SYRK_PIPE == 2
    double Xc[NQ];
    XCoef c1;
    {
      const XCoef c0 = genX_a(0, g, cl);
      if (NP > 1) c1 = genX_a(1 < NP ? 1 : 0, g, cl);
      genX_b(0, c0, Xc);
    }
#pragma unroll
    for (int pp = 0; pp < NP; ++pp) {
      XCoef c2 = c1;
      if (pp + 2 < NP) c2 = genX_a(pp + 2 < NP ? pp + 2 : 0, g, cl);
      double Xn[NQ];
      if (pp + 1 < NP) genX_b(pp + 1 < NP ? pp + 1 : 0, c1, Xn);
#pragma unroll
      for (int ti = 0; ti < NQ; ++ti)
#pragma unroll
        for (int tj = 0; tj <= ti; ++tj) T[tri(ti, tj)] = UPPER_H ? mfma(Xc[tj], Xc[ti], T[tri(ti, tj)])
                                                                : mfma(Xc[ti], Xc[tj], T[tri(ti, tj)]);
      if (pp + 1 < NP) {
        // the step's LDS reads behind the first MFMAs, its VALU after them
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
        for (int r = 2; r < NT; ++r) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, SOCP_SYRK_V, 0);
        }
      }
      SCHED_FENCE();
      c1 = c2;
#pragma unroll
      for (int q = 0; q < NQ; ++q) Xc[q] = Xn[q];
    }
#elif SOCP_SYRK_PIPE
    // software-pipelined: row step pp+1 of X is generated (LDS coefficient
    // reads, AGPR reads of G, FMAs) while the MFMAs of step pp run, one MFMA
    // between every few of those instructions
    double Xc[NQ];
    genX(0, Xc);
#pragma unroll
    for (int pp = 0; pp < NP; ++pp) {
      double Xn[NQ];
      if (pp + 1 < NP) genX(pp + 1, Xn);
#pragma unroll
      for (int ti = 0; ti < NQ; ++ti)
#pragma unroll
        for (int tj = 0; tj <= ti; ++tj) T[tri(ti, tj)] = UPPER_H ? mfma(Xc[tj], Xc[ti], T[tri(ti, tj)])   // block (tj, ti)
                                                                : mfma(Xc[ti], Xc[tj], T[tri(ti, tj)]);  // block (ti, tj)
      if (pp + 1 < NP) {
#pragma unroll
        for (int r = 0; r < NT; ++r) {
          __builtin_amdgcn_sched_group_barrier(0x008, SOCP_SYRK_M, 0);  // one MFMA,
          __builtin_amdgcn_sched_group_barrier(0x100, SOCP_SYRK_L, 0);  // two LDS reads,
          __builtin_amdgcn_sched_group_barrier(0x002, SOCP_SYRK_V, 0);  // eight VALU (measured: 1/1/3 -0.7 %)
        }
      }
      SCHED_FENCE();
#pragma unroll
      for (int q = 0; q < NQ; ++q) Xc[q] = Xn[q];
    }
#else
#pragma unroll
    for (int pp = 0; pp < NP; ++pp) {
      double X[NQ];
      genX(pp, X);
#pragma unroll
      for (int ti = 0; ti < NQ; ++ti)
#pragma unroll
        for (int tj = 0; tj <= ti; ++tj) T[tri(ti, tj)] = UPPER_H ? mfma(X[tj], X[ti], T[tri(ti, tj)]) : mfma(X[ti], X[tj], T[tri(ti, tj)]);
      if (pp % 2 == 1) SCHED_FENCE();
    }
#endif
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
            for (int tj = 0; tj <= ti; ++tj) T[tri(ti, tj)] = UPPER_H ? mfma(Aq[tj], Aq[ti], T[tri(ti, tj)]) : mfma(Aq[ti], Aq[tj], T[tri(ti, tj)]);
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

  // ------------------------------------------------- H^-1 by a block sweep
  // The inverse Li = H^-1 of densesolver.jl:47-48 (cholesky! + potrs(I)) is
  // formed by a symmetric Gauss-Jordan sweep with 16x16 pivot tiles P; after
  // every tile is swept the lower tiles hold -H^-1.  Per tile:
  //   D = M_PP = L L' (its current Schur complement), W = L^-1 (VALU, below);
  //   Y_i = W M_Pi                      (i != P, MFMA)
  //   M_ij -= Y_i' Y_j                  (i, j != P: the Schur update in Gram
  //                                      form, as accurate as a Cholesky step)
  //   M_Pi <- W' Y_i = D^-1 M_Pi, M_PP <- -W'W = -D^-1          (MFMA)
  // Every pivot of D is a Cholesky pivot of H (a Schur complement), so a
  // pivot <= 0 or NaN fails exactly where LAPACK potrf fails inside
  // cholesky!.  C/D-tile algebra: lane (g, cl) holds X[g+4r][cl] in register
  // r, so register s of a tile is the k-step-s operand of mfma_f64_16x16x4,
  // and sum_s mfma(U[s], V[s]) = U'V for any two tiles U, V.

  // sum_s mfma(U[s], V[s], C) with the NEG modifiers of gfx950 f64 MFMA
  // (blgp bit 0 negates A, bit 2 negates C)
  template <int NEG>
  __device__ __forceinline__ static d4 mm(const d4& U, const d4& V, d4 C) {
#pragma unroll
    for (int s = 0; s < 4; ++s) C = __builtin_amdgcn_mfma_f64_16x16x4f64(U[s], V[s], C, 0, 0, NEG);
    return C;
  }

  // tile transpose: by MFMA against the identity (X' I), no LDS hand-off, or
  // through LDS
  __device__ __forceinline__ d4 ttrans(const d4& X, const d4& Id) {
#if SOCP_TRANSPOSE_MFMA
    return mm<0>(X, Id, (d4){0.0, 0.0, 0.0, 0.0});
#else
    return transpose(X);
#endif
  }

#ifndef SOCP_SWEEP_LOOKAHEAD
#define SOCP_SWEEP_LOOKAHEAD 1
#endif
  // The MFMA work of panel P that the next pivot tile's factorisation does not
  // wait for: the Gram updates other than tile (P+1, P+1), the new panel tiles
  // M_Pi and M_PP.  Enumerated at compile time so it can be dealt out between
  // the row blocks of the next factorisation (look-ahead).
  struct PanelOp {
    int kind, i, j;  // 0: M_ij -= Y_i'Y_j, 1: new panel tile i, 2: M_PP = -W'W, -1: none
  };
  template <int Q, int P>
  static constexpr PanelOp panel_op(int idx) {
    int cnt = 0;
    for (int i = 0; i < Q; ++i)
      for (int j = 0; j <= i; ++j) {
        if (i == P || j == P || (i == P + 1 && j == P + 1)) continue;
        if (cnt++ == idx) return PanelOp{0, i, j};
      }
    for (int i = 0; i < Q; ++i) {
      if (i == P) continue;
      if (cnt++ == idx) return PanelOp{1, i, 0};
    }
    if (cnt++ == idx) return PanelOp{2, P, P};
    return PanelOp{-1, 0, 0};
  }
  template <int Q, int P>
  static constexpr int panel_op_count() {
    int c = 0;
    while (panel_op<Q, P>(c).kind >= 0) ++c;
    return c;
  }
  template <int Q, int P, int OP>
  __device__ __forceinline__ static void do_panel_op(d4 (&M)[Q * (Q + 1) / 2], const d4 (&Y)[Q], const d4& W) {
    constexpr PanelOp o = panel_op<Q, P>(OP);
    const d4 z = (d4){0.0, 0.0, 0.0, 0.0};
    if constexpr (o.kind == 0) {
      M[tri(o.i, o.j)] = mm<1>(Y[o.i], Y[o.j], M[tri(o.i, o.j)]);  // -= Y_i'Y_j
    } else if constexpr (o.kind == 1) {
      if constexpr (o.i < P) M[tri(P, o.i)] = mm<0>(W, Y[o.i], z);  // W'Y_i = D^-1 M_Pi
      else M[tri(o.i, P)] = mm<0>(Y[o.i], W, z);                    // its transpose
    } else if constexpr (o.kind == 2) {
      M[tri(P, P)] = mm<1>(W, W, z);  // -W'W = -D^-1
    }
  }
  template <int Q, int P, int LO, int HI>
  __device__ __forceinline__ static void do_panel_ops(d4 (&M)[Q * (Q + 1) / 2], const d4 (&Y)[Q], const d4& W) {
    if constexpr (LO < HI) {
      do_panel_op<Q, P, LO>(M, Y, W);
      do_panel_ops<Q, P, LO + 1, HI>(M, Y, W);
    }
  }
  // hook for the next factorisation: after row block B, a quarter of the ops
  template <int Q, int P>
  struct PanelHook {
    d4 (&M)[Q * (Q + 1) / 2];
    const d4 (&Y)[Q];
    const d4& W;
    template <int B>
    __device__ __forceinline__ void run() const {
      constexpr int N = panel_op_count<Q, P>();
      do_panel_ops<Q, P, (N * B) / 4, (N * (B + 1)) / 4>(M, Y, W);
    }
  };

  // Panel P of the sweep, given W = L^-1 of its pivot tile (factored by the
  // previous panel, overlapped with that panel's MFMA work).
  template <int Q, bool SUBST, int P>
  __device__ __forceinline__ void sweep_panel(d4 (&M)[Q * (Q + 1) / 2], const d4& Id, const d4& W, bool& ok) {
    MARK_BEGIN("sweep_tiles");
    if constexpr (P < Q) {
      d4 X[Q];  // M_Pi in C/D layout (stored transposed below the pivot tile)
#pragma unroll
      for (int i = P + 1; i < Q; ++i) X[i] = ttrans(M[tri(i, P)], Id);
      const d4 WT = ttrans(W, Id);
      const d4 z = (d4){0.0, 0.0, 0.0, 0.0};
      d4 Y[Q];
#pragma unroll
      for (int i = 0; i < Q; ++i)
        if (i != P) Y[i] = mm<0>(WT, i < P ? M[tri(P, i)] : X[i], z);  // W M_Pi
      STAMP_SUB(2);
      if constexpr (P + 1 < Q) {
        // the next pivot tile first, then its factorisation with the rest of
        // this panel's MFMA work dealt out between its row blocks
        M[tri(P + 1, P + 1)] = mm<1>(Y[P + 1], Y[P + 1], M[tri(P + 1, P + 1)]);
        d4 Wn;
#if SOCP_SWEEP_LOOKAHEAD
        factor_tile<TILE_INPL>(M[tri(P + 1, P + 1)], Wn, ok, PanelHook<Q, P>{M, Y, W});
#else
        do_panel_ops<Q, P, 0, panel_op_count<Q, P>()>(M, Y, W);
        factor_tile<TILE_INPL>(M[tri(P + 1, P + 1)], Wn, ok);
#endif
        STAMP_SUB(1);
        sweep_panel<Q, SUBST, P + 1>(M, Id, Wn, ok);
      } else {
        do_panel_ops<Q, P, 0, panel_op_count<Q, P>()>(M, Y, W);
        STAMP_SUB(3);
      }
    }
  }
  template <int Q, bool SUBST>
  __device__ __forceinline__ void sweep_tiles(d4 (&M)[Q * (Q + 1) / 2], const d4& Id, bool& ok) {
    d4 W;
    factor_tile<TILE_INPL>(M[tri(0, 0)], W, ok);
    STAMP_SUB(0);
    sweep_panel<Q, SUBST, 0>(M, Id, W, ok);
  }

  // Symmetric sweep of every pivot of M (lower tiles; padding rows carry an
  // identity diagonal, so sweeping them is harmless): leaves -M^-1.
  template <int Q, bool SUBST>
  __device__ __forceinline__ bool sweep(d4 (&M)[Q * (Q + 1) / 2]) {
    LANE_IDS();
    d4 Id;
#pragma unroll
    for (int r = 0; r < 4; ++r) Id[r] = (g + 4 * r == cl) ? 1.0 : 0.0;
    bool ok = true;
    sweep_tiles<Q, SUBST>(M, Id, ok);
    return ok;
  }

  // ------------------------------------ H = L L' by 16x16 tiles (CHOL shapes)
  // densesolver.jl:47 cholesky!(Hermitian(H)), right-looking by tile panels.
  // The explicit Li of :48 is never formed: ALi = A Li enters as Z = L^-1 A'
  // (S = A Li A' = Z'Z, :49-50) and Li v as two triangular solves.  Storage:
  // the SYRK leaves block (i, j), i <= j, of H in T[tri(j, i)] (upper tiles),
  // so the panel row U_Pi needs no transpose; after panel P, T[tri(P, P)]
  // holds W_P = L_PP^-1 (factor_tile) and T[tri(i, P)] = L_iP' (i > P).
  // Panel P: Y_i = W_P U_Pi = L_iP' (MFMA), U_ij -= Y_i'Y_j (P < i <= j).
  // Look-ahead: Y_{P+1} and U_{P+1,P+1} first, then the next pivot tile is
  // factored with the rest of the panel's MFMA work -- and the panel's tile
  // row of Z -- dealt out between its row blocks.  Every pivot is a Cholesky
  // pivot of H (potrf's test, as the sweep's).
  struct CholOp {
    int kind, i, j;  // 0: Y_i = W_P U_Pi, 1: U_ij -= Y_i'Y_j, 2: the Z row of panel P, -1: none
  };
  template <int P>
  static constexpr CholOp chol_op(int idx) {
    int cnt = 0;
    for (int i = P + 2; i < NQ; ++i)
      if (cnt++ == idx) return CholOp{0, i, 0};
    for (int j = P + 1; j < NQ; ++j)  // column-major: U_{P+1,P+2} and U_{P+2,P+2} (the next panel's) first
      for (int i = P + 1; i <= j; ++i) {
        if (i == P + 1 && j == P + 1) continue;
        if (cnt++ == idx) return CholOp{1, i, j};
      }
    if (cnt++ == idx) return CholOp{2, P, 0};
    return CholOp{-1, 0, 0};
  }
  template <int P>
  static constexpr int chol_op_count() {
    int c = 0;
    while (chol_op<P>(c).kind >= 0) ++c;
    return c;
  }
  // Z_P = W_P (A'_P - sum_{Q<P} L_PQ Z_Q) (left-looking: one accumulator tile),
  // S += Z_P'Z_P (Sv[0]); Z' row-major in LDS at O_AL (where the sweep path
  // keeps A Li): Z'[c][j] = LDS(O_AL + c*LDA + j).
  template <int P>
  __device__ __forceinline__ void z_row(const d4& WT) {
    LANE_IDS();
    SYNC();
    d4 acc;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = LDS(O_A + cl * LDA + 16 * P + g + 4 * r);  // A'[16P+g+4r][cl]
#pragma unroll
    for (int Q = 0; Q < P; ++Q) {
      d4 Zq;
#pragma unroll
      for (int r = 0; r < 4; ++r) Zq[r] = LDS(O_AL + cl * LDA + 16 * Q + g + 4 * r);
      acc = mm<1>(T[tri(P, Q)], Zq, acc);  // -= L_PQ Z_Q
    }
    const d4 Z = mm<0>(WT, acc, (d4){0.0, 0.0, 0.0, 0.0});
    Sv[0] = mm<0>(Z, Z, Sv[0]);
#pragma unroll
    for (int r = 0; r < 4; ++r) LDS(O_AL + cl * LDA + 16 * P + g + 4 * r) = Z[r];
  }
  template <int P, int OP>
  __device__ __forceinline__ void chol_op_run(const d4& WT) {
    constexpr CholOp o = chol_op<P>(OP);
    if constexpr (o.kind == 0) {
      T[tri(o.i, P)] = mm<0>(WT, T[tri(o.i, P)], (d4){0.0, 0.0, 0.0, 0.0});
    } else if constexpr (o.kind == 1) {
      T[tri(o.j, o.i)] = mm<1>(T[tri(o.i, P)], T[tri(o.j, P)], T[tri(o.j, o.i)]);
    } else if constexpr (o.kind == 2) {
      z_row<P>(WT);
    }
  }
  template <int P, int LO, int HI>
  __device__ __forceinline__ void chol_ops(const d4& WT) {
    if constexpr (LO < HI) {
      chol_op_run<P, LO>(WT);
      chol_ops<P, LO + 1, HI>(WT);
    }
  }
  template <int P>
  struct CholHook {
    Small& s;
    const d4& WT;
    template <int B>
    __device__ __forceinline__ void run() const {
      constexpr int N = chol_op_count<P>();
      s.template chol_ops<P, (N * B) / 4, (N * (B + 1)) / 4>(WT);
    }
  };
  template <int P>
  __device__ __forceinline__ void chol_panel(const d4& W, bool& ok) {
    if constexpr (P < NQ) {
      MARK_BEGIN("chol_panel");
      const d4 WT = transpose(W);
      if constexpr (P + 1 < NQ) {
        T[tri(P + 1, P)] = mm<0>(WT, T[tri(P + 1, P)], (d4){0.0, 0.0, 0.0, 0.0});
        T[tri(P + 1, P + 1)] = mm<1>(T[tri(P + 1, P)], T[tri(P + 1, P)], T[tri(P + 1, P + 1)]);
        d4 Wn;
        factor_tile<TILE_INPL>(T[tri(P + 1, P + 1)], Wn, ok, CholHook<P>{*this, WT});
        T[tri(P, P)] = W;
        chol_panel<P + 1>(Wn, ok);
      } else {
        z_row<P>(WT);
        T[tri(P, P)] = W;
      }
    }
  }
  __device__ __forceinline__ bool chol() {
    if (SOCP_KO & 131072) {
      LANE_IDS();
#pragma unroll
      for (int r = 0; r < 4; ++r) Sv[0][r] = (g + 4 * r == cl) ? 1.0 : 0.0;
      return true;
    }
    Sv[0] = (d4){0.0, 0.0, 0.0, 0.0};
    bool ok = true;
    d4 W;
    factor_tile<TILE_INPL>(T[tri(0, 0)], W, ok);
    chol_panel<0>(W, ok);
    SYNC();
    return ok;
  }

  // ---------------- the explicit inverse from the Cholesky factor (chol_inv)
  // densesolver.jl:47-48: Li = H^-1 from cholesky!(H), the reference's
  // ldiv!(Li, fact, I) -- H = L L', then Li = L^-T L^-1 -- on 16x16 tiles:
  // (1) H = L L' right-looking by tile panels as chol() does it (its look-ahead:
  //     the next pivot tile factored with the panel's other MFMA work dealt out
  //     between its row blocks), leaving M[tri(P, P)] = W_P = L_PP^-1 and
  //     M[tri(i, P)] = L_iP' (i > P); every pivot is potrf's (status 2 / 3);
  // (2) Y = L^-1 in place, row by row: Y_PP = W_P,
  //     Y_ab = -W_a sum_{b <= q < a} L_aq Y_qb (a > b);
  // (3) Li = Y'Y in place, row by row: Li_ab = sum_{q >= a} Y_qa' Y_qb (a >= b),
  //     symmetric by construction.
  // In: M in the upper-block form (M[tri(j, i)] = block (i, j), i <= j, the
  // SYRK's UPPER_H output); out: the lower tiles of the inverse in the natural
  // C/D layout (M[tri(a, b)] = block (a, b)), as symv and the record read them.
  struct GCholOp {
    int kind, i, j;  // 0: M_iP = W_P M_iP (= L_iP'), 1: M_ij -= L_iP L_jP', -1: none
  };
  template <int Q, int P>
  static constexpr GCholOp gchol_op(int idx) {
    int cnt = 0;
    for (int i = P + 2; i < Q; ++i)
      if (cnt++ == idx) return GCholOp{0, i, 0};
    for (int j = P + 1; j < Q; ++j)
      for (int i = P + 1; i <= j; ++i) {
        if (i == P + 1 && j == P + 1) continue;
        if (cnt++ == idx) return GCholOp{1, i, j};
      }
    return GCholOp{-1, 0, 0};
  }
  template <int Q, int P>
  static constexpr int gchol_op_count() {
    int c = 0;
    while (gchol_op<Q, P>(c).kind >= 0) ++c;
    return c;
  }
  template <int Q, int P, int LO, int HI>
  __device__ __forceinline__ static void gchol_ops(d4 (&M)[Q * (Q + 1) / 2], const d4& WT) {
    if constexpr (LO < HI) {
      constexpr GCholOp o = gchol_op<Q, P>(LO);
      if constexpr (o.kind == 0)
        M[tri(o.i, P)] = mm<0>(WT, M[tri(o.i, P)], (d4){0.0, 0.0, 0.0, 0.0});
      else
        M[tri(o.j, o.i)] = mm<1>(M[tri(o.i, P)], M[tri(o.j, P)], M[tri(o.j, o.i)]);
      gchol_ops<Q, P, LO + 1, HI>(M, WT);
    }
  }
  template <int Q, int P>
  struct GCholHook {
    d4 (&M)[Q * (Q + 1) / 2];
    const d4& WT;
    template <int B>
    __device__ __forceinline__ void run() const {
      constexpr int N = gchol_op_count<Q, P>();
      gchol_ops<Q, P, (N * B) / 4, (N * (B + 1)) / 4>(M, WT);
    }
  };
  template <int Q, int P>
  __device__ __forceinline__ void gchol_panel(d4 (&M)[Q * (Q + 1) / 2], const d4& W, bool& ok) {
    if constexpr (P < Q) {
      MARK_BEGIN("chol_inv_panel");
      if constexpr (P + 1 < Q) {
        const d4 WT = transpose(W);
        M[tri(P + 1, P)] = mm<0>(WT, M[tri(P + 1, P)], (d4){0.0, 0.0, 0.0, 0.0});
        M[tri(P + 1, P + 1)] = mm<1>(M[tri(P + 1, P)], M[tri(P + 1, P)], M[tri(P + 1, P + 1)]);
        d4 Wn;
        factor_tile<TILE_INPL>(M[tri(P + 1, P + 1)], Wn, ok, GCholHook<Q, P>{M, WT});
        M[tri(P, P)] = W;
        gchol_panel<Q, P + 1>(M, Wn, ok);
      } else {
        M[tri(P, P)] = W;
      }
    }
  }
  template <int Q>
  __device__ __forceinline__ bool chol_inv(d4 (&M)[Q * (Q + 1) / 2]) {
    MARK_BEGIN("chol_inv");
    const d4 z = (d4){0.0, 0.0, 0.0, 0.0};
    bool ok = true;
    {
      d4 W;
      factor_tile<TILE_INPL>(M[tri(0, 0)], W, ok);
      gchol_panel<Q, 0>(M, W, ok);
    }
    // Y = L^-1: row a reads rows q < a of Y (done) and row a of L from column b up
#pragma unroll
    for (int a = 1; a < Q; ++a) {
      const d4 WTa = transpose(M[tri(a, a)]);
#pragma unroll
      for (int b = 0; b < a; ++b) {
        d4 S = mm<0>(M[tri(a, b)], M[tri(b, b)], z);  // L_ab W_b
#pragma unroll
        for (int q = b + 1; q < a; ++q) S = mm<0>(M[tri(a, q)], M[tri(q, b)], S);  // + L_aq Y_qb
        M[tri(a, b)] = mm<1>(WTa, S, z);  // -W_a S
      }
    }
    // Li = Y'Y: tile (a, b) is the last reader of Y_ab (row-major order)
#pragma unroll
    for (int a = 0; a < Q; ++a)
#pragma unroll
      for (int b = 0; b <= a; ++b) {
        d4 acc = z;
#pragma unroll
        for (int q = a; q < Q; ++q) acc = mm<0>(M[tri(q, a)], M[tri(q, b)], acc);
        M[tri(a, b)] = acc;
      }
    return ok;
  }

  // the transpose buffer, when it lives in dead k-vectors, is zeroed again at
  // the end of a factorisation: their padding rows [k, KP) are never written
  // by the solves and must read as zero (G'T2 reads them against G's zero rows)
  __device__ __forceinline__ void clear_tb() {
    if constexpr (SH::TB_ALIAS) {
      SYNC();
      for (int e = lane; e < 16 * 17; e += 64) LDS(O_TB + e) = 0.0;
      SYNC();
    }
  }
  __device__ __forceinline__ d4 transpose(d4 t) {
    MARK_BEGIN("transpose");
    LANE_IDS();
    SYNC();
#pragma unroll
    for (int r = 0; r < 4; ++r) LDS(O_TB + (g + 4 * r) * 17 + cl) = t[r];
    SYNC();
    d4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = LDS(O_TB + cl * 17 + g + 4 * r);
    return o;
  }

  __device__ __forceinline__ void dump_sym(double* out, bool upper = false) {
#pragma unroll
    for (int ti = 0; ti < NQ; ++ti)
#pragma unroll
      for (int tj = 0; tj <= ti; ++tj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int R = (upper ? 16 * tj : 16 * ti) + g + 4 * r, Cc = (upper ? 16 * ti : 16 * tj) + cl;
          if (R < n && Cc < n) {
            out[R * n + Cc] = T[tri(ti, tj)][r];
            if (ti != tj) out[Cc * n + R] = T[tri(ti, tj)][r];
          }
        }
  }

  // H (+A'A) -> sweep -> Li;  ALi' = Li A' (n x m);  S = A ALi';  S^-1.
  __device__ __forceinline__ int factor(bool identity, bool addAA) {
    MARK_BEGIN("factor");
    LANE_IDS();
    STAMP(SP_OTHER);
    if (!identity && !(SOCP_KO & 4)) compute_U();
    STAMP(SP_U);
    form_H(addAA);
    SYNC();
    STAMP(SP_SYRK);
#ifdef SOCP_DIAG
    // diagnostic dump per problem: H, H^-1 (n x n each), lam, wbar (k each), Li A' (n x m), S (m x m)
    double* dbg = (a.dbg && a.mode == MODE_KKT) ? a.dbg + dbg_p * (int64_t)(2 * n * n + 2 * k + n * m + m * m) : nullptr;
    if (dbg && !CHOL) dump_sym(dbg, UPPER_H);
#endif
    if constexpr (CHOL) {
      const bool okH = chol();
      STAMP(SP_SWEEP_H);
      if (!okH) {
        clear_tb();
        return ST_CHOL_H;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (g + 4 * r == cl && cl >= m) Sv[0][r] = 1.0;
#if SOCP_S_TILE
      // S = L L' on one tile (potrf's pivot test), S^-1 = W'W with W = L^-1:
      // one MFMA tile chain and four MFMAs instead of the 16-pivot sweep
      bool okS = true;
      if (!(SOCP_KO & 8)) {
        d4 Ws;
        factor_tile<TILE_INPL>(Sv[0], Ws, okS);
        Sv[0] = mm<0>(Ws, Ws, (d4){0.0, 0.0, 0.0, 0.0});
      }
      clear_tb();
      STAMP(SP_SCHUR);
      if (!okS) return ST_CHOL_S;
#else
      const bool okS = (SOCP_KO & 8) ? true : sweep<1, false>(Sv);
      clear_tb();
      STAMP(SP_SCHUR);
      if (!okS) return ST_CHOL_S;
      Sv[0] = -Sv[0];
#endif
      return 0;
    }
    bool okH;
    if constexpr (INV_CHOL) {
      okH = chol_inv<NQ>(T);
    } else {
      okH = sweep<NQ, true>(T);
    }
    STAMP(SP_SWEEP_H);
    if (!okH) {
      clear_tb();
      return ST_CHOL_H;
    }
    if constexpr (!INV_CHOL) {
#pragma unroll
      for (int t = 0; t < NT; ++t) T[t] = -T[t];  // the sweep leaves -H^-1
    }
#ifdef SOCP_DIAG
    if (dbg) {
      dump_sym(dbg + n * n);
      for (int i = lane; i < k; i += 64) {
        dbg[2 * n * n + i] = LDS(LAM + i);
        dbg[2 * n * n + k + i] = LDS(WB + i);
      }
    }
#endif
    // S = A Li A' (densesolver.jl:49-50: ALi = A*Li, S = ALi*A'), one 16-column
    // tile of Li A' at a time: it lives only here, the solves use A (Li n0).
#pragma unroll
    for (int tq = 0; tq < MQ; ++tq) {
      d4 ALc[NQ];
#pragma unroll
      for (int ti = 0; ti < NQ; ++ti) {
        d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int tk = 0; tk < NQ; ++tk) {
          d4 Ut;
          if (tk >= ti)
            Ut = T[tri(tk, ti)];
          else
            Ut = transpose(T[tri(ti, tk)]);
#pragma unroll
          for (int s = 0; s < 4; ++s) acc = mfma(Ut[s], LDS(O_A + (16 * tq + cl) * LDA + 16 * tk + g + 4 * s), acc);
        }
        ALc[ti] = acc;
      }
#ifdef SOCP_DIAG
      if (dbg) {
        double* dA = dbg + 2 * n * n + 2 * k;
#pragma unroll
        for (int ti = 0; ti < NQ; ++ti)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int R = 16 * ti + g + 4 * r, Cc = 16 * tq + cl;
            if (R < n && Cc < m) dA[R * m + Cc] = ALc[ti][r];
          }
      }
#endif
#pragma unroll
      for (int tm = tq; tm < MQ; ++tm) {
        d4 acc = (d4){0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int tk = 0; tk < NQ; ++tk)
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            const double av = LDS(O_A + (16 * tm + cl) * LDA + 16 * tk + g + 4 * s);
            // INV_CHOL: block (tq, tm) of S, the upper-block form chol_inv reads
            acc = INV_CHOL ? mfma(ALc[tk][s], av, acc) : mfma(av, ALc[tk][s], acc);
          }
        Sv[tri(tm, tq)] = acc;
      }
      if constexpr (KEEP_AL) {
#pragma unroll
        for (int ti = 0; ti < NQ; ++ti) AL[tq][ti] = transpose(ALc[ti]);  // A Li = (Li A')'
      } else if constexpr (AL_LDS) {
        // A Li row-major in LDS: lane (g, cl) holds (A Li)[16tq+cl][16ti+g+4r]
#pragma unroll
        for (int ti = 0; ti < NQ; ++ti)
#pragma unroll
          for (int r = 0; r < 4; ++r) LDS(O_AL + (16 * tq + cl) * LDA + 16 * ti + g + 4 * r) = ALc[ti][r];
      }
    }
#pragma unroll
    for (int tm = 0; tm < MQ; ++tm)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int R = 16 * tm + g + 4 * r, Cc = 16 * tm + cl;
        if (R == Cc && R >= m) Sv[tri(tm, tm)][r] = 1.0;
      }
#ifdef SOCP_DIAG
    if (dbg) {
      double* dS = dbg + 2 * n * n + 2 * k + n * m;
#pragma unroll
      for (int tm = 0; tm < MQ; ++tm)
#pragma unroll
        for (int tq = 0; tq <= tm; ++tq)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int R = (INV_CHOL ? 16 * tq : 16 * tm) + g + 4 * r, Cc = (INV_CHOL ? 16 * tm : 16 * tq) + cl;
            if (R < m && Cc < m) dS[R * m + Cc] = dS[Cc * m + R] = Sv[tri(tm, tq)][r];
          }
    }
#endif
    SYNC();
    bool okS;
    if constexpr (INV_CHOL) {
      okS = chol_inv<MQ>(Sv);
    } else {
      okS = sweep<MQ, false>(Sv);
    }
    clear_tb();  // the sweeps' and A Li's transposes ran in the dead k-vectors (TB_ALIAS)
    STAMP(SP_SCHUR);
    if (!okS) return ST_CHOL_S;
    if constexpr (!INV_CHOL) {
#pragma unroll
      for (int t = 0; t < MT; ++t) Sv[t] = -Sv[t];
    }
    return 0;
  }

  // out = M*v for a symmetric matrix stored as lower tiles (C/D layout).
  // Lower part: per tile row, reduce over the 16 column lanes; strictly upper
  // part (transposed off-diagonal tiles): reduce over the 4 row groups.
  template <int Q>
  __device__ __forceinline__ void symv(const d4 (&M)[Q * (Q + 1) / 2], int vin, int vout) {
    MARK_BEGIN("symv");
    LANE_IDS();
    double vc[Q], P2[Q];
#pragma unroll
    for (int t = 0; t < Q; ++t) {
      vc[t] = LDS(vin + 16 * t + cl);
      P2[t] = 0.0;
    }
    double P1row[Q];
#pragma unroll
    for (int ti = 0; ti < Q; ++ti) {
      double vr[4], P1[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        vr[r] = LDS(vin + 16 * ti + g + 4 * r);
        double acc = 0.0;
#pragma unroll
        for (int tj = 0; tj <= ti; ++tj) acc = fma(M[tri(ti, tj)][r], vc[tj], acc);
        P1[r] = acc;
      }
#pragma unroll
      for (int tj = 0; tj < ti; ++tj)
#pragma unroll
        for (int r = 0; r < 4; ++r) P2[tj] = fma(M[tri(ti, tj)][r], vr[r], P2[tj]);
      int base = 0;
      rs16<4, 8>(P1, cl, base);  // one value per lane: row 16ti + g + 4*base
      P1row[ti] = P1[0] + 0.0 * base;
      // stash the row index in base via the lane's own cl bits (see write below)
    }
    if constexpr (Q > 1) {
#pragma unroll
      for (int t = 0; t < Q; ++t) P2[t] = rows_sum(P2[t]);
    }
    SYNC();
    {
      // rs16<4,8>: bit 8 of cl picks entries 2-3, bit 4 picks the odd one; masks
      // 2 and 1 are all-reduce steps, so the lane holds entry (cl>>3&1)*2 + (cl>>2&1)
      const int r = ((cl >> 3) & 1) * 2 + ((cl >> 2) & 1);
#pragma unroll
      for (int ti = 0; ti < Q; ++ti) LDS(vout + 16 * ti + g + 4 * r) = P1row[ti];
    }
    SYNC();
    if constexpr (Q > 1) {  // one tile has no strictly upper part
      if (g == 0) {
#pragma unroll
        for (int t = 0; t < Q; ++t) LDS(vout + 16 * t + cl) += P2[t];
      }
      SYNC();
    }
  }

  // symv<1> with v in column layout in registers (vc = v[cl], every lane); out
  // to LDS as symv's, and in registers in row layout, yr[s] = out[g + 4s]
  __device__ __forceinline__ void symv1_r(const d4& M, double vc, int vout, double (&yr)[4]) {
    MARK_BEGIN("symv");
    LANE_IDS();
    double P1[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) P1[r] = fma(M[r], vc, 0.0);
    int base = 0;
    rs16<4, 8>(P1, cl, base);  // row g + 4 (cl >> 2)
    LDS(vout + g + 4 * (cl >> 2)) = P1[0];
    yr[0] = dpp_all<0x150>(P1[0]);
    yr[1] = dpp_all<0x154>(P1[0]);
    yr[2] = dpp_all<0x158>(P1[0]);
    yr[3] = dpp_all<0x15C>(P1[0]);
  }

  // Triangular solves against chol()'s factor (T[tri(P, P)] = W_P = L_PP^-1,
  // T[tri(i, P)] = L_iP').  Tile products alternate between the two vector
  // layouts of a C/D tile, so no LDS round trip sits on the chain: W v
  // (v[cl] in every lane of column cl) gives (W v)[g+4r] after a 16-lane
  // all-reduce; M'u (u[g+4r] in the lanes of row group g) gives (M'u)[cl]
  // after the four-row sum.  The off-diagonal products of earlier tiles are
  // accumulated lane-locally and reduced once per tile.
#ifndef SOCP_ALLRED_RS
#define SOCP_ALLRED_RS 1
#endif
  __device__ __forceinline__ static void allred16(double (&v)[4]) {
#if SOCP_ALLRED_RS
    // reduce-scatter (entry r ends in lanes 4r..4r+3 of the row: rs16's base is
    // cl >> 2), then each entry broadcast from lane 4r by row_newbcast: 9 DPP
    // moves and 6 adds per 64-bit lane value instead of 16 and 16
    LANE_IDS();
    int base = 0;
    rs16<4, 8>(v, cl, base);
    const double t = v[0];
    v[0] = dpp_all<0x150>(t);
    v[1] = dpp_all<0x154>(t);
    v[2] = dpp_all<0x158>(t);
    v[3] = dpp_all<0x15C>(t);
#else
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += row_partner<8>(v[r]);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += row_partner<4>(v[r]);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += row_partner<2>(v[r]);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += row_partner<1>(v[r]);
#endif
  }
  // out = L^-1 v: t_P = W_P (v_P - sum_{Q<P} L_PQ t_Q).  rc: v in column
  // layout (every lane holds v[16i+cl]); tv: t in row layout (tv[P][r] =
  // t[16P+g+4r] in every lane of row group g), for a product that takes its
  // operand in that layout without the LDS round trip.
  __device__ __forceinline__ void trsv_fwd_r(const double (&rc)[NQ], int vout, double (&tv)[NQ][4]) {
    MARK_BEGIN("trsv_fwd");
    LANE_IDS();
    double pa[NQ];  // lane partials of sum_Q L_iQ t_Q
#pragma unroll
    for (int i = 0; i < NQ; ++i) pa[i] = 0.0;
#pragma unroll
    for (int P = 0; P < NQ; ++P) {
      const double rp = P > 0 ? rc[P] - rows_sum(pa[P]) : rc[P];
      double t4[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) t4[r] = T[tri(P, P)][r] * rp;
      allred16(t4);  // t_P[g+4r]
#pragma unroll
      for (int i = P + 1; i < NQ; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) pa[i] = fma(T[tri(i, P)][r], t4[r], pa[i]);
      if (cl < 4) LDS(vout + 16 * P + g + 4 * cl) = cl == 0 ? t4[0] : (cl == 1 ? t4[1] : (cl == 2 ? t4[2] : t4[3]));
#pragma unroll
      for (int r = 0; r < 4; ++r) tv[P][r] = t4[r];
    }
    SYNC();
  }
  // out = L^-T v: x_P = W_P' (v_P - sum_{i>P} L_iP' x_i); in place is allowed.
  // xs: x in column layout (every lane holds x[16P+cl]).
  __device__ __forceinline__ void trsv_bwd(int vin, int vout, double (&xs)[NQ]) {
    MARK_BEGIN("trsv_bwd");
    LANE_IDS();
    double ur[NQ][4], pa[NQ][4];  // v (row layout), lane partials of sum_i L_iP' x_i
#pragma unroll
    for (int P = 0; P < NQ; ++P)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        ur[P][r] = LDS(vin + 16 * P + g + 4 * r);
        pa[P][r] = 0.0;
      }
#pragma unroll
    for (int P = NQ - 1; P >= 0; --P) {
      double u4[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) u4[r] = pa[P][r];
      if (P < NQ - 1) allred16(u4);
      double acc = 0.0;
#pragma unroll
      for (int r = 0; r < 4; ++r) acc = fma(T[tri(P, P)][r], P < NQ - 1 ? ur[P][r] - u4[r] : ur[P][r], acc);
      const double x = rows_sum(acc);  // x_P[cl]
      xs[P] = x;
#pragma unroll
      for (int Q = 0; Q < P; ++Q)
#pragma unroll
        for (int r = 0; r < 4; ++r) pa[Q][r] = fma(T[tri(P, Q)][r], x, pa[Q][r]);
    }
    SYNC();
    if (g == 0) {
#pragma unroll
      for (int P = 0; P < NQ; ++P) LDS(vout + 16 * P + cl) = xs[P];
    }
    SYNC();
  }

  // out[row] = (G u)[row] + add1[row] - add2[row] for rows < k (u in column layout).
  // Rows are reduced over the 16 column lanes in chunks of up to 8 row-steps.
  template <int P0, int CH, bool NEG = false>
  __device__ __forceinline__ void gemv_G_chunk(const double (&uq)[NQ], int add1, int add2, int out) {
    LANE_IDS();
    constexpr int CF = RSCount<CH, 8>::value;
    // the addends of the rows this lane ends up holding, read before the products
    double a1[CF], a2[CF];
    {
      const int b0 = rs16_base<CH, 8>(cl);
#pragma unroll
      for (int j = 0; j < CF; ++j) {
        const int row = 4 * (P0 + b0 + j) + g;  // < KP: in the k-vector
        a1[j] = add1 >= 0 ? LDS(add1 + row) : 0.0;
        a2[j] = LDS(add2 + row);
      }
    }
    double P[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      double acc = 0.0;
      {
        double gr[NQ];
        a_get_row<NQ>(G[P0 + j], gr);
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc = fma(gr[q], uq[q], acc);
      }
      P[j] = acc;
    }
    int base = 0;
    rs16<CH, 8>(P, cl, base);
#pragma unroll
    for (int j = 0; j < CF; ++j) {
      const int row = 4 * (P0 + base + j) + g;
      if (row < k) {
        double v = P[j];
        if (add1 >= 0) v = v + a1[j];
        v = v - a2[j];
        LDS(out + row) = NEG ? -v : v;
      }
    }
    if constexpr (P0 + CH < NP) {
      constexpr int NXT = (NP - P0 - CH) < 8 ? (NP - P0 - CH) : 8;
      gemv_G_chunk<P0 + CH, NXT, NEG>(uq, add1, add2, out);
    }
  }
  __device__ __forceinline__ void gemv_G(int u, int add1, int add2, int out) {
    MARK_BEGIN("gemv_G");
    LANE_IDS();
    double uq[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) uq[q] = LDS(u + 16 * q + cl);
    gemv_G_chunk<0, (NP < 8 ? NP : 8)>(uq, add1, add2, out);
    SYNC();
  }
  // the same with u in column layout in registers (uq[q] = u[16q+cl]); NEG:
  // store the negated rows
  template <bool NEG = false>
  __device__ __forceinline__ void gemv_G_r(const double (&uq)[NQ], int add1, int add2, int out) {
    MARK_BEGIN("gemv_G");
    gemv_G_chunk<0, (NP < 8 ? NP : 8), NEG>(uq, add1, add2, out);
    SYNC();
  }

  // acc[q] (all lanes) = (G' v)[16q+cl].  The v reads of the next batch of
  // row steps are issued before the current batch's products (one exposed
  // LDS round trip per call, not one per pair of row steps).  hook.run<b>()
  // runs inside batch b's scheduling region (b < 2): independent work whose
  // latency the batch's VALU stream hides (resid_scaling).
  struct NoGtHook {
    template <int B>
    __device__ __forceinline__ void run() {}
  };
  template <class HK = NoGtHook>
  __device__ __forceinline__ void gemv_Gt(int v, double (&acc)[NQ], HK&& hook = HK()) {
    MARK_BEGIN("gemv_Gt");
    LANE_IDS();
    constexpr int VB = 8;
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = 0.0;
    double vb[VB];
#pragma unroll
    for (int j = 0; j < VB; ++j) vb[j] = j < NP ? LDS(v + 4 * j + g) : 0.0;
#pragma unroll
    for (int p0 = 0; p0 < NP; p0 += VB) {
      double vn[VB];
#pragma unroll
      for (int j = 0; j < VB; ++j) vn[j] = p0 + VB + j < NP ? LDS(v + 4 * (p0 + VB + j) + g) : 0.0;
      SCHED_FENCE();
      if (p0 == 0) hook.template run<0>();
      if (p0 == VB) hook.template run<1>();
#pragma unroll
      for (int j = 0; j < VB; ++j) {
        if (p0 + j < NP) {
          {
            double gr[NQ];
            a_get_row<NQ>(G[p0 + j < NP ? p0 + j : 0], gr);
#pragma unroll
            for (int q = 0; q < NQ; ++q) acc[q] = fma(gr[q], vb[j], acc[q]);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < VB; ++j) vb[j] = vn[j];
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      acc[q] = rows_sum(acc[q]);
    }
  }

#ifndef SOCP_LDS_BATCH
#define SOCP_LDS_BATCH 16  // LDS reads issued per round trip in the A products (8 where HOIST_CST is off)
#endif
  static constexpr int LDB = HOIST_CST ? SOCP_LDS_BATCH : 8;
  static constexpr int AMB = (NQ * 4) % LDB == 0 ? LDB : 4;
  static constexpr int ATB = (MQ * 4) % (LDB / NQ > 0 ? LDB / NQ : 1) == 0 ? (LDB / NQ > 0 ? LDB / NQ : 1) : 1;
  // acc[q] (all lanes) = (A' v)[16q+cl]: rows split over the 4 lane groups
  // vr (optional): v in registers, vr[s] = v[g + 4s] (s < 4 MQ), instead of LDS
  __device__ __forceinline__ void At_mv(int v, double (&acc)[NQ], int base = O_A, const double* vr = nullptr) {
    MARK_BEGIN("At_mv");
    LANE_IDS();
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = 0.0;
    // the reads of a step batch issued before its products (one LDS round
    // trip per SOCP_LDS_BATCH rows, not one per row: the scheduler otherwise
    // interleaves read, wait, fma)
#pragma unroll
    for (int s0 = 0; s0 < MQ * 4; s0 += ATB) {
      double vi[ATB], av[ATB][NQ];
#pragma unroll
      for (int s = 0; s < ATB; ++s) {
        const int i = g + 4 * (s0 + s);
        vi[s] = vr ? vr[s0 + s] : LDS(v + i);
#pragma unroll
        for (int q = 0; q < NQ; ++q) av[s][q] = LDS(base + i * LDA + 16 * q + cl);
      }
      SCHED_FENCE();
#pragma unroll
      for (int s = 0; s < ATB; ++s)
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc[q] = fma(av[s][q], vi[s], acc[q]);
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      acc[q] = rows_sum(acc[q]);
    }
  }
  // out[i] = (A u)[i] - sub[i] for i < m (columns split over the 4 lane groups);
  // returns sum of out[i]^2 on lanes g == 0
  __device__ __forceinline__ double A_mv(int u, int sub, int out, int base = O_A, bool neg = false) {
    MARK_BEGIN("A_mv");
    LANE_IDS();
    double sq = 0.0;
#pragma unroll
    for (int tm = 0; tm < MQ; ++tm) {
      const int i = 16 * tm + cl;
      double acc = 0.0;
#pragma unroll
      for (int t0 = 0; t0 < NQ * 4; t0 += AMB) {
        double av[AMB], uv[AMB];
#pragma unroll
        for (int t = 0; t < AMB; ++t) {
          av[t] = LDS(base + i * LDA + g + 4 * (t0 + t));
          uv[t] = LDS(u + g + 4 * (t0 + t));
        }
        SCHED_FENCE();
#pragma unroll
        for (int t = 0; t < AMB; ++t) acc = fma(av[t], uv[t], acc);
      }
      acc = rows_sum(acc);
      if (g == 0 && i < m) {
        const double v = acc - LDS(sub + i);
        LDS(out + i) = neg ? -v : v;
        sq = fma(v, v, sq);
      }
    }
    return sq;
  }

  // A_mv with u in row layout in registers (tv[P][r] = u[16P+g+4r], trsv_fwd_r's
  // output): the same products in the same order
  // (mc: the result in column layout in every lane, mc[tm] = out[16 tm + cl],
  // 0 for rows >= m)
  __device__ __forceinline__ double A_mv_r(const double (&tv)[NQ][4], int sub, int out, int base, double (&mc)[MQ]) {
    MARK_BEGIN("A_mv");
    LANE_IDS();
    double sq = 0.0;
#pragma unroll
    for (int tm = 0; tm < MQ; ++tm) {
      const int i = 16 * tm + cl;
      const double sb = LDS(sub + i);
      double acc = 0.0;
#pragma unroll
      for (int t0 = 0; t0 < NQ * 4; t0 += AMB) {
        double av[AMB];
#pragma unroll
        for (int t = 0; t < AMB; ++t) av[t] = LDS(base + i * LDA + g + 4 * (t0 + t));
        SCHED_FENCE();
#pragma unroll
        for (int t = 0; t < AMB; ++t) acc = fma(av[t], tv[(t0 + t) >> 2][(t0 + t) & 3], acc);
      }
      acc = rows_sum(acc);
      const double v = acc - sb;
      if (g == 0 && i < m) {
        LDS(out + i) = v;
        sq = fma(v, v, sq);
      }
      mc[tm] = i < m ? v : 0.0;
    }
    return sq;
  }

  // rd = A'y + G'z + c, rp = Ax - b, rz = Gx + s - h (solver.jl:109-118)
  __device__ __forceinline__ void residuals(double& nd, double& np_, double& gap) {
    MARK_BEGIN("residuals");
    LANE_IDS();
    double acc[NQ], at[NQ];
    // the small operands read up front, in one round trip: c and x (column
    // layout), z and s (slot layout)
    constexpr int NS = KP > 64 ? 2 : 1;
    double cq[NQ], xq[NQ], zv[NS], sv[NS];
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      cq[q] = LDS(C_ + 16 * q + cl);
      xq[q] = LDS(X_ + 16 * q + cl);
    }
#pragma unroll
    for (int t = 0; t < NS; ++t) {
      zv[t] = LDS(Z_ + 64 * t + lane);
      sv[t] = LDS(S_ + 64 * t + lane);
    }
    if (SOCP_KO & 32) {
      for (int q = 0; q < NQ; ++q) acc[q] = 0.0;
    } else {
      gemv_Gt(Z_, acc);
    }
    if (SOCP_KO & 128) {
      for (int q = 0; q < NQ; ++q) at[q] = 0.0;
    } else {
      At_mv(Y_, at);
    }
    double d2 = 0.0, zs = 0.0;
    if (g == 0) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int j = 16 * q + cl;
        if (j < n) {
          const double v = (at[q] + acc[q]) + cq[q];
          LDS(RD + j) = -v;  // the residuals are stored negated: the affine RHS (solver.jl:124)
          d2 = fma(v, v, d2);
        }
      }
    }
    const double p2 = (SOCP_KO & 128) ? 0.0 : A_mv(X_, B_, RP, O_A, true);
    if (!(SOCP_KO & 16)) gemv_G_r<true>(xq, S_, H_, DZ);
#pragma unroll
    for (int t = 0; t < NS; ++t)
      if (64 * t + lane < k) zs += zv[t] * sv[t];
    if (SOCP_KO & 64) {
      nd = np_ = gap = d2 + p2 + zs;
    } else {
      double r3[3] = {d2, p2, zs};  // the three whole-wave sums in one interleaved scan
      dpp_scan<3>(r3, lane, 0, false);
      nd = sqrt(readlane_d(r3[0], 63));
      np_ = sqrt(readlane_d(r3[1], 63));
      gap = readlane_d(r3[2], 63);
    }
  }

  // The matrix part of solve_kkt(::DenseSolver) (densesolver.jl:66-85), between
  // the cone ops: n0 = GWiWi*k2 + dx (+A'dy if sing); m0 = ALi*n0 - dy, taken as
  // A*(Li*n0) - dy; cy = S^-1 m0; m0 = sing ? dy - cy : -cy (init: -cy);
  // n0 += A'm0; cx = Li n0; k1 = G cx - k2.   In: RD RP T2(=W^-2 k2) K2.  Out: RX RY K1.
  __device__ __forceinline__ void solve_matrix_part(bool init) {
    MARK_BEGIN("solve_matrix_part");
    LANE_IDS();
    // n0 in column layout, in every lane (the CHOL path hands it to trsv_fwd_r
    // in registers; the sweep path's symv reads it from N0)
    double n0[NQ];
    {
      double acc[NQ], at[NQ];
      if (SOCP_KO & 512) {
        for (int q = 0; q < NQ; ++q) acc[q] = LDS(T2 + 16 * q + cl);
      } else {
        gemv_Gt(T2, acc);
      }
      if (sing) At_mv(RP, at);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        const int j = 16 * q + cl;
        double v = acc[q] + LDS(RD + j);
        if (sing) v = v + at[q];
        n0[q] = v;
      }
      if (!CHOL && g == 0) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) LDS(N0 + 16 * q + cl) = n0[q];
      }
    }
    if constexpr (!CHOL) SYNC();
    STAMP_X(4);
    double tv[NQ][4];  // t = L^-1 n0 in row layout (CHOL)
    double cxr[NQ];    // cx in column layout (CHOL: trsv_bwd's output)
    if constexpr (CHOL) {
      if (SOCP_KO & 256) {
        if (g == 0)
          for (int q = 0; q < NQ; ++q) LDS(TN + 16 * q + cl) = n0[q];
        SYNC();
        for (int P = 0; P < NQ; ++P)
          for (int r = 0; r < 4; ++r) tv[P][r] = LDS(TN + 16 * P + g + 4 * r);
      } else {
        trsv_fwd_r(n0, TN, tv);  // t = L^-1 n0
      }
    } else
      symv<NQ>(T, N0, TN);   // Li n0
    STAMP_X(5);
    // CHOL with one S tile: m0, cy and the next m0 stay in registers
    constexpr bool MREG = CHOL && MQ == 1;
    double m0c[MQ], m0r[4];
    if (SOCP_KO & 2048) {
      for (int j = lane; j < m; j += 64) LDS(M0 + j) = LDS(TN + j);
    } else if constexpr (CHOL)
      A_mv_r(tv, RP, M0, O_AL, m0c);  // m0 = A Li n0 - dy = Z't - dy
    else if constexpr (AL_LDS)
      A_mv(N0, RP, M0, O_AL);  // m0 = (A Li) n0 - dy: no wait for Li n0
    else
      A_mv(TN, RP, M0);        // m0 = A (Li n0) - dy
    if constexpr (MREG) {
      if (SOCP_KO & 2048) {
        SYNC();
        for (int j = lane; j < m; j += 64) LDS(RY + j) = LDS(M0 + j);
        SYNC();
        for (int s = 0; s < 4; ++s) m0r[s] = LDS(RY + g + 4 * s);
      } else {
        double rp[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) rp[s] = LDS(RP + g + 4 * s);
        symv1_r(Sv[0], m0c[0], RY, m0r);  // cy = S^-1 m0
#pragma unroll
        for (int s = 0; s < 4; ++s)
          m0r[s] = g + 4 * s < m ? ((sing && !init) ? rp[s] - m0r[s] : -m0r[s]) : 0.0;
      }
    } else {
      SYNC();
      if (SOCP_KO & 2048) {
        for (int j = lane; j < m; j += 64) LDS(RY + j) = LDS(M0 + j);
        SYNC();
      } else {
        symv<MQ>(Sv, M0, RY);  // cy = S^-1 m0
      }
      if (lane < m) LDS(M0 + lane) = (sing && !init) ? LDS(RP + lane) - LDS(RY + lane) : -LDS(RY + lane);
      SYNC();
    }
    STAMP_X(6);
    if constexpr (KEEP_AL) {
      // cx = Li (n0 + A'm0) = Li n0 + (A Li)' m0
      ALt_mv(M0, TN, RX);
    } else if constexpr (AL_LDS) {
      // cx = Li (n0 + A'm0) = Li n0 + (A Li)' m0: one Li product per solve
      // (CHOL: cx = L^-T (t + Z m0))
      double at[NQ], tn[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) tn[q] = LDS(TN + 16 * q + cl);  // read with At_mv's operands
      if (SOCP_KO & 2048) {
        for (int q = 0; q < NQ; ++q) at[q] = 0.0;
      } else {
        At_mv(M0, at, O_AL, MREG ? m0r : nullptr);
      }
      if (g == 0) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) LDS(RX + 16 * q + cl) = tn[q] + at[q];
      }
      SYNC();
      if constexpr (CHOL) {
        if (!(SOCP_KO & 256)) {
          trsv_bwd(RX, RX, cxr);
        } else {
#pragma unroll
          for (int q = 0; q < NQ; ++q) cxr[q] = LDS(RX + 16 * q + cl);
        }
      }
      STAMP_X(7);
    } else {
      double at[NQ];
      At_mv(M0, at);
      if (g == 0) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) LDS(N0 + 16 * q + cl) = LDS(N0 + 16 * q + cl) + at[q];
      }
      SYNC();
      symv<NQ>(T, N0, RX);  // cx = Li n0
    }
    if (SOCP_KO & 1024) {
      for (int i = lane; i < k; i += 64) LDS(K1 + i) = LDS(RX + (i & 63)) - LDS(K2 + i);
      SYNC();
    } else if constexpr (CHOL) {
      gemv_G_r(cxr, -1, K2, K1);  // cx from trsv_bwd's registers
    } else {
      gemv_G(RX, -1, K2, K1);
    }
  }

  // out[j] = add[j] + ((A Li)' v)[j]: per tile column, an in-lane sum over the
  // tile's rows (registers) and the four row groups (rows_sum)
  __device__ __forceinline__ void ALt_mv(int v, int add, int out) {
    LANE_IDS();
    double vr[MQ][4];
#pragma unroll
    for (int tq = 0; tq < MQ; ++tq)
#pragma unroll
      for (int r = 0; r < 4; ++r) vr[tq][r] = LDS(v + 16 * tq + g + 4 * r);
#pragma unroll
    for (int ti = 0; ti < NQ; ++ti) {
      double acc = 0.0;
#pragma unroll
      for (int tq = 0; tq < MQ; ++tq)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc = fma(AL[KEEP_AL ? tq : 0][KEEP_AL ? ti : 0][r], vr[tq][r], acc);
      acc = rows_sum(acc);
      if (g == 0) LDS(out + 16 * ti + cl) = acc + LDS(add + 16 * ti + cl);
    }
    SYNC();
  }

  // ------------------------------------------------------- factor record
  // setup_iter's products for the later solve_kkt calls: H^-1 and S^-1 in
  // register-tile (lane) order, the scaling vectors and per-cone constants the
  // solves read, and `sing` (densesolver.jl:41-52 keeps them in the solver
  // object; here one record per problem in HBM).
  static __device__ constexpr int rec_kv(int v) {
    return v == 0 ? KV_LAM : v == 1 ? KV_WB : v == 2 ? KV_CA : v == 3 ? KV_CB : KV_IL;
  }
  static constexpr int64_t REC_SING = (int64_t)(NT + MT) * 256 + 5 * KP + 20 * NCS + (AL_LDS ? MPAD * LDA : 0);
  static constexpr int64_t REC_STATUS = REC_SING + 1;  // setup_iter's status, read first by solve_kkt
  __device__ __forceinline__ void store_record(int64_t p) {
    LANE_IDS();
    double* r = a.rec + p * a.rec_stride;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) r[(t * 4 + q) * 64 + lane] = T[t][q];
    r += NT * 256;
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) r[(t * 4 + q) * 64 + lane] = Sv[t][q];
    r += MT * 256;
#pragma unroll
    for (int v = 0; v < 5; ++v)
      for (int i = lane; i < KP; i += 64) r[v * KP + i] = LDS(kvs(rec_kv(v)) + i);
    r += 5 * KP;
    for (int i = lane; i < 20 * NCS; i += 64) r[i] = LDS(O_CC + i);
    if constexpr (AL_LDS)
      for (int i = lane; i < MPAD * LDA; i += 64) r[20 * NCS + i] = LDS(O_AL + i);
    if (lane == 0) r[REC_SING - (NT + MT) * 256 - 5 * KP] = sing ? 1.0 : 0.0;  // REC_SING
  }
  __device__ __forceinline__ void load_record(int64_t p) {
    LANE_IDS();
    const double* r = a.rec + p * a.rec_stride;
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) T[t][q] = r[(t * 4 + q) * 64 + lane];
    r += NT * 256;
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) Sv[t][q] = r[(t * 4 + q) * 64 + lane];
    r += MT * 256;
#pragma unroll
    for (int v = 0; v < 5; ++v)
      for (int i = lane; i < KP; i += 64) LDS(kvs(rec_kv(v)) + i) = r[v * KP + i];
    r += 5 * KP;
    for (int i = lane; i < 20 * NCS; i += 64) LDS(O_CC + i) = r[i];
    if constexpr (AL_LDS)
      for (int i = lane; i < MPAD * LDA; i += 64) LDS(O_AL + i) = r[20 * NCS + i];
    sing = uni(r[REC_SING - (NT + MT) * 256 - 5 * KP]) != 0.0;
    SYNC();
  }

  // ------------------------------------------------------------- driver
  // solve_socp (solver.jl:40-153) as a micro-phase loop.  solve_kkt
  // (densesolver.jl:54-90) is MP_SOLVE_HEAD -> MP_SOLVE_MAT -> MP_SOLVE_TAIL;
  // `ret` says which solve it is (init, KKT entry, affine, combined).
  // KM = 0: the solver kernel (MODE_SOLVE); KM = 1: the plugin-entry kernel
  // (MODE_KKT, MODE_SETUP, MODE_SOLVEKKT), compiled apart so the solver's
  // register allocation does not carry the entry paths.
  template <int KM>
  __device__ __forceinline__ void run(int64_t p) {
    const int mode = KM ? a.mode : (a.mode == MODE_KKT ? (int)MODE_KKT : (int)MODE_SOLVE);
    STAMP(SP_LOAD);
    dbg_p = p;
    int status = ST_MAXIT, iters = 0, it = 0;
    double nd = NAN, np_ = NAN, gap = NAN;
    double ll = 0.0;
    bool fac_ident = false, fac_aa = false, dm_aa = false;
    int fret = 0, ret = 0, fst = 0;
    int after_singtest;
    bool have_sing = false;
    if (mode == MODE_SOLVEKKT) {  // setup_iter failed for this problem: NaN solution, its status
      const int st0 = (int)uni(a.rec[p * a.rec_stride + REC_STATUS]);
      if (st0) {
        for (int j = lane; j < n; j += 64) a.cx[p * n + j] = NAN;
        for (int i = lane; i < m; i += 64) a.cy[p * m + i] = NAN;
        for (int i = lane; i < k; i += 64) {
          a.cz[p * k + i] = NAN;
          a.cs[p * k + i] = NAN;
        }
        if (lane == 0) a.status[p] = st0;
        return;
      }
    }
    if (mode == MODE_KKT || mode == MODE_SETUP || mode == MODE_SOLVEKKT) {
      for (int i = lane; i < k; i += 64) {
        if (mode != MODE_SOLVEKKT) {
          LDS(S_ + i) = a.s[p * k + i];
          LDS(Z_ + i) = a.z[p * k + i];
        }
        if (mode != MODE_SETUP) {
          LDS(DZ + i) = a.dz[p * k + i];
          LDS(DS + i) = a.ds[p * k + i];
        }
      }
      if (mode != MODE_SETUP) {
        for (int j = lane; j < n; j += 64) LDS(RD + j) = a.dx[p * n + j];
        for (int i = lane; i < m; i += 64) LDS(RP + i) = a.dy[p * m + i];
      }
      after_singtest = MP_KKT;
      if (mode == MODE_SOLVEKKT) {  // solve_kkt against the setup_iter record
        load_record(p);
        have_sing = true;
        after_singtest = MP_SOLVE_HEAD;
        ret = RET_KKT;
      }
    } else if (a.flags & F_WARM) {
      for (int j = lane; j < n; j += 64) LDS(X_ + j) = a.x[p * n + j];
      for (int i = lane; i < m; i += 64) LDS(Y_ + i) = a.y[p * m + i];
      for (int i = lane; i < k; i += 64) {
        LDS(Z_ + i) = a.z[p * k + i];
        LDS(S_ + i) = a.s[p * k + i];
      }
      after_singtest = MP_ITER;
    } else {
      after_singtest = MP_INIT;
    }
    SYNC();
    int phase;
    if (have_sing) {
      phase = after_singtest;
    } else if (a.sing) {
      sing = uni((int)a.sing[p]) != 0;
      phase = after_singtest;
    } else {
      sing = false;
      phase = MP_SINGTEST;
    }
    bool done = false;
    while (!done) {
      LANE_IDS();
      if (KM && phase == MP_SAVE) {  // setup_iter done: keep the factorisation for the solves
        // (outside the switch: the solver kernel's phase switch is left as it
        // was tuned -- an extra case there re-lays the loop and costs ~4%)
        store_record(p);
        status = 0;
        break;
      }
      int next = phase;
      switch (phase) {
        case MP_SINGTEST:  // Problem's `sing` (Socp.jl:49-56): is G'G positive definite?
          MARK_BEGIN("case MP_SINGTEST");
          scaling_identity();
          fac_ident = true;
          fac_aa = false;
          fret = MP_SINGTEST_POST;
          next = MP_FACTOR;
          break;
        case MP_SINGTEST_POST:
          MARK_BEGIN("case MP_SINGTEST_POST");
          sing = (fst == ST_CHOL_H);
          next = after_singtest;
          break;
        case MP_FACTOR:  // setup_iter (densesolver.jl:41-52)
          MARK_BEGIN("case MP_FACTOR");
          fst = factor(fac_ident, fac_aa);
          if (fst && fret != MP_SINGTEST_POST) {
            status = fst;
            done = true;
          }
          next = fret;
          break;
        case MP_INIT:  // initial point: the KKT system with W = I (solver.jl:68-84)
          MARK_BEGIN("case MP_INIT");
          scaling_identity();
          for (int j = lane; j < n; j += 64) LDS(RD + j) = -LDS(C_ + j);
          for (int i = lane; i < m; i += 64) LDS(RP + i) = LDS(B_ + i);
          for (int i = lane; i < k; i += 64) {
            LDS(DZ + i) = LDS(H_ + i);
            LDS(DS + i) = 0.0;
          }
          SYNC();
          fac_ident = true;
          fac_aa = sing;
          fret = MP_SOLVE_HEAD;
          ret = RET_INIT;
          next = MP_FACTOR;
          break;
        case MP_ITER: {  // residuals (solver.jl:109-118), compute_scaling (:106), exit test (:122)
          MARK_BEGIN("case MP_ITER");
          STAMP(SP_OTHER);
          // after the last iteration the reference loop ends without another
          // residual evaluation (solver.jl:105-151): they are formed then only
          // when the caller asked for the final residual norms
          if (it >= a.maxit && !a.res) {
            done = true;
            break;
          }
          bool dm;
          if constexpr (SOCP_RESID_SCAL && !(SOCP_KO & (2 | 4096))) {
            // (after the last iteration the scaling is computed too, and unused)
            dm = resid_scaling(nd, np_, gap, ll, dm_aa);
            STAMP(SP_RESID);
            if (it >= a.maxit) {
              done = true;
              break;
            }
          } else {
            if (SOCP_KO & 2) {
              nd = np_ = gap = 1.0;
            } else {
              residuals(nd, np_, gap);
            }
            STAMP(SP_RESID);
            if (it >= a.maxit) {
              done = true;
              break;
            }
            dm = scaling_op(ll, dm_aa, true);
          }
          STAMP(SP_VOP);
          if (dm) {
            status = ST_DOMAIN;
            done = true;
            break;
          }
          if (nd + np_ + gap < a.tol) {
            status = ST_CONVERGED;
            done = true;
            break;
          }
          // (rmul!(dx, -1) etc., solver.jl:124: the residuals and ds were stored negated)
          fac_ident = false;
          fac_aa = sing;
          fret = MP_SOLVE_HEAD;
          ret = RET_AFFINE;
          next = MP_FACTOR;
          break;
        }
        case MP_KKT: {
          MARK_BEGIN("case MP_KKT");
          const bool dm = scaling_op(ll, dm_aa, false);
          if (dm) {
            status = ST_DOMAIN;
            done = true;
            break;
          }
          fac_ident = false;
          fac_aa = sing;
          fret = mode == MODE_SETUP ? MP_SAVE : MP_SOLVE_HEAD;
          ret = RET_KKT;
          next = MP_FACTOR;
          break;
        }
        case MP_SOLVE_HEAD: {
          // a solve (densesolver.jl:54-90) -- head, matrix part, tail -- and,
          // after the affine one, the combined one: without trips through the
          // phase dispatch (each costs ~1 %)
          for (;;) {
            MARK_BEGIN("case MP_SOLVE_HEAD");
            STAMP(SP_OTHER);
            solve_head();
            STAMP(SP_VOP);
            MARK_BEGIN("case MP_SOLVE_MAT");
            solve_matrix_part(ret == RET_INIT);
            STAMP(SP_SOLVE);
            MARK_BEGIN("case MP_SOLVE_TAIL");
            const bool do_step = ret == RET_AFFINE || ret == RET_COMBINED;
            int dom = 0;
            const double tstep = solve_tail(do_step, dm_aa, dom);
            STAMP(SP_VOP);
            if (ret == RET_KKT) {
              status = 0;
              for (int j = lane; j < n; j += 64) a.cx[p * n + j] = LDS(RX + j);
              for (int i = lane; i < m; i += 64) a.cy[p * m + i] = LDS(RY + i);
              for (int i = lane; i < k; i += 64) {
                a.cz[p * k + i] = LDS(RZ + i);
                a.cs[p * k + i] = LDS(RS + i);
              }
              done = true;
              break;
            }
            if (ret == RET_INIT) {  // cone shift (solver.jl:86-104)
              double alphp, alphd;  // max_step(-iz), max_step(iz)
              maxstep_op(RZ, alphp, alphd);
              for (int j = lane; j < n; j += 64) LDS(X_ + j) = LDS(RX + j);
              for (int i = lane; i < m; i += 64) LDS(Y_ + i) = LDS(RY + i);
              for (int i = lane; i < k; i += 64) {
                const double iz = LDS(RZ + i), e = e_of(i);
                LDS(S_ + i) = (fabs(alphp) < a.init_eps) ? -iz : -iz + (1.0 + alphp) * e;
                LDS(Z_ + i) = (fabs(alphd) < a.init_eps) ? iz : iz + (1.0 + alphd) * e;
              }
              SYNC();
              next = MP_ITER;
              break;
            }
            if (dom) {
              status = ST_DOMAIN;
              done = true;
              break;
            }
            if (ret == RET_AFFINE) {  // centering + corrector, then the combined solve
              affine_post(tstep, ll);
              STAMP(SP_STEP);
              ret = RET_COMBINED;
              continue;
            }
            // combined direction: step and update (solver.jl:143-150)
            const double stp = tstep * a.step;
            {  // every read first (n, m <= 64, k <= 128 here), then the updates
              constexpr int NS = KP > 64 ? 2 : 1;
              const int ly = lane < MPAD ? lane : 0;
              const double xo = LDS(X_ + lane), rx = LDS(RX + lane), yo = LDS(Y_ + ly), ry = LDS(RY + ly);
              double zo[NS], rz[NS], so[NS], rs[NS];
#pragma unroll
              for (int t = 0; t < NS; ++t) {
                const int i = 64 * t + lane;
                zo[t] = LDS(Z_ + i);
                rz[t] = LDS(RZ + i);
                so[t] = LDS(S_ + i);
                rs[t] = LDS(RS + i);
              }
              if (lane < n) LDS(X_ + lane) = xo + rx * stp;
              if (lane < m) LDS(Y_ + lane) = yo + ry * stp;
#pragma unroll
              for (int t = 0; t < NS; ++t) {
                const int i = 64 * t + lane;
                if (i < k) {
                  LDS(Z_ + i) = zo[t] + rz[t] * stp;
                  LDS(S_ + i) = so[t] + rs[t] * stp;
                }
              }
            }
            SYNC();
            STAMP(SP_STEP);
            iters = ++it;
            next = MP_ITER;
            break;
          }
          break;
        }
        default:
          done = true;
          break;
      }
      if (done) break;
      phase = uni(next);
    }
    if (mode != MODE_SOLVE) {
      if (lane == 0) a.status[p] = status;
      if (mode == MODE_SETUP && lane == 0) a.rec[p * a.rec_stride + REC_STATUS] = (double)status;
      SYNC();
      STAMP(SP_STORE);
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
    STAMP(SP_STORE);
#ifdef SOCP_DIAG
    if (lane == 0) reinterpret_cast<unsigned long long*>(socp_lds + O_STAMPS)[NSTAMP] += iters;
#endif
  }

  __device__ __forceinline__ void flush_stamps() {
#ifdef SOCP_DIAG
    SYNC();
    if (lane == 0 && a.stamps) {
      const unsigned long long* st = reinterpret_cast<const unsigned long long*>(socp_lds + O_STAMPS);
      for (int i = 0; i <= NSTAMP + NSUBSTAMP; ++i) atomicAdd(a.stamps + i, st[i]);
    }
#endif
  }
};

// KM bit 0: the plugin-entry kernel (MODE_KKT / MODE_SETUP / MODE_SOLVEKKT)
// instead of the solver; bit 1: the explicit-inverse variant (XI above)
template <int NQ, int NP, int MQ, int KM>
#ifndef SOCP_DEV_MINW
#define SOCP_DEV_MINW 1  // probe builds only: waves per SIMD the register allocation must allow
#endif
__global__ void __launch_bounds__(64, KM == 0 ? SOCP_DEV_MINW : 1) socp_small_kernel(SmallArgs args) {
  Small<NQ, NP, MQ, (KM & 2) != 0> S(args);
  S.init_tables();
  STAMP_START_S(S);
  while (true) {
    int p = 0;
    if (threadIdx.x == 0) p = atomicAdd(args.counter, 1);
    p = __shfl(p, 0);
    if ((int64_t)p >= args.B) break;
    S.load_problem(p);
    S.template run<KM & 1>(p);
  }
  S.flush_stamps();
}

}  // namespace socp
