// socp_kernels.hpp — internal launch interface between socp_api.hip and the
// kernels: the register-resident instantiations (gen_inst.py) and the blocked
// kernel (socp_large.hip).
#pragma once
#include <hip/hip_runtime.h>
#include "socp_small.hpp"

namespace socp {

struct SmallVariant {
  int NQ, NP, MQ;
  const void* kernel;  // socp_small_kernel<NQ,NP,MQ,0>: MODE_SOLVE
  const char* name;
  const void* kkt_kernel;  // socp_small_kernel<NQ,NP,MQ,1>: MODE_KKT / MODE_SETUP / MODE_SOLVEKKT
  const char* kkt_name;
  // SOCP_F_EXPLICIT_INVERSE (KM 2 / 3): the same two with Li = H^-1 formed by
  // the sweep; NULL where the shape sweeps anyway (m > 16)
  const void* xi_kernel;
  const char* xi_name;
  const void* xi_kkt_kernel;
  const char* xi_kkt_name;
};

// table of compiled register-resident variants, ordered by (NQ, NP, MQ)
const SmallVariant* small_variants(int* count);

// ------------------------------------------------------- blocked kernel
// socp_large.hip: one 512-thread workgroup per problem, the problem's vectors
// in LDS, its matrices in a per-workgroup slot of an HBM workspace.
constexpr int LARGE_NB_MAX = 8;  // NPAD, MPAD <= 512: a swept panel row lives in registers
// NPAD <= 2048 where H is factored (the default, not SOCP_F_EXPLICIT_INVERSE):
// panels wider than 512 are factored in windows (socp_large.hip panel_chol_wide)
constexpr int LARGE_NB_MAX_CHOL = 32;
// k bound of the blocked kernel: its LDS / vector offsets and the row offsets
// into X (KP x NPAD) are 32-bit ints (socp_api.hip large_fits)
constexpr int LARGE_KMAX = 1 << 21;

struct LargeLayout {
  int NPAD, MPAD, KP, RW;  // n, m rounded up to 64, k to 16; RW = max(NPAD, MPAD)
  // LDS offsets (doubles)
  int o_rc, o_cc, o_kvd, o_kvl, o_nv, o_mv, o_row, o_rv, o_part, o_red, o_fx, total;
  int sy;  // 1: the staged SYRK's four chunk buffers fit (socp_large.hip form_H_staged_g)
  // workspace-slot offsets (doubles)
  int64_t w_x, w_h, w_ap, w_at, w_yp, w_rv, w_t, w_s, w_v, w_lv, w_total;
  // per-problem factor record (socp_dense handles): what solve_kkt reads
  int64_t r_h, r_ap, r_at, r_t, r_s, r_v, r_total;
};
__host__ __device__ inline int64_t large_al(int64_t v) { return (v + 31) / 32 * 32; }
__host__ __device__ inline LargeLayout large_layout(int n, int m, int k) {
  LargeLayout L;
  L.NPAD = (n + 63) / 64 * 64;
  L.MPAD = ((m > 0 ? m : 1) + 63) / 64 * 64;
  L.KP = (k + 15) / 16 * 16;
  L.RW = L.NPAD > L.MPAD ? L.NPAD : L.MPAD;
  // The region from 0 holds what is dead while a factorisation runs -- seven
  // k-vectors (RZ RS K0 K1 K2 T1 T2) and the sweep / solve scratch -- so the
  // staged SYRK's four 4-row X chunk buffers (4 NPAD doubles each, written by
  // LDS-DMA, whose destination must lie in the first 64 KiB) can overlay it,
  // padded up to 16 NPAD when NPAD is 256 or 512 and the LDS allows.
  for (int pass = 0; pass < 2; ++pass) {
    const bool want = pass == 0 && (L.NPAD == 256 || L.NPAD == 512);
    int o = 0;
    L.o_kvd = o;  o += 7 * L.KP;      // dead k-vectors
    L.o_row = o;  o += 2 * L.RW > 1024 ? 2 * L.RW : 1024;  // sweep: pivot rows / four 16x16 tile slots
    L.o_rv = o;   o += 64;            // sweep: -1/d of the panel's pivots
    L.o_part = o; o += 8 * L.MPAD;    // A x partial sums per wavefront
    if (want && o < 16 * L.NPAD) o = 16 * L.NPAD;
    L.o_kvl = o;  o += 8 * L.KP;      // live k-vectors (H Z S DZ DS LAM WB CA)
    L.o_rc = o;   o += L.KP;          // element code: cone*4 + type
    L.o_cc = o;   o += 12 * MAXC;     // per-cone constants CC_*
    L.o_nv = o;   o += 6 * L.NPAD;    // n-vectors
    L.o_mv = o;   o += 5 * L.MPAD;    // m-vectors
    L.o_red = o;  o += 64;            // block reductions (slot 63: the next problem index)
    L.o_fx = o;   o += 8 * 64;        // W^-1 G fast path: per wavefront, per-cone sums and heads
    L.total = o;
    L.sy = want ? 1 : 0;
    if (!want || (long)o * 8 + 64 <= 160 * 1024) break;
  }
  int64_t w = 0;
  L.w_x = w;  w += large_al((int64_t)L.KP * L.NPAD);    // X = W^-1 G
  L.w_h = w;  w += large_al((int64_t)L.NPAD * L.NPAD);  // H -> Li
  L.w_ap = w; w += large_al((int64_t)L.MPAD * L.NPAD);  // A, column-major
  L.w_at = w; w += large_al((int64_t)L.NPAD * L.MPAD);  // A, row-major
  L.w_yp = w; w += large_al((int64_t)L.RW * L.RW);      // sweep pivot rows, 64 x RW per panel
  L.w_rv = w; w += large_al((int64_t)L.RW);             // sweep: -1/d of every pivot
  L.w_t = w;  w += large_al((int64_t)L.NPAD * L.MPAD);  // Li A'
  L.w_s = w;  w += large_al((int64_t)L.MPAD * L.MPAD);  // S -> S^-1
  L.w_v = w;  w += large_al(3 * (int64_t)L.KP + 12 * MAXC + 8);  // LAM WB CA, CC_*, sing, status
  L.w_lv = w; w += large_al(L.total);  // the vectors themselves when they exceed the LDS (GV kernels)
  L.w_total = w;
  w = 0;
  L.r_h = w;  w += large_al((int64_t)L.NPAD * L.NPAD);
  L.r_ap = w; w += large_al((int64_t)L.MPAD * L.NPAD);
  L.r_at = w; w += large_al((int64_t)L.NPAD * L.MPAD);
  L.r_t = w;  w += large_al((int64_t)L.NPAD * L.MPAD);
  L.r_s = w;  w += large_al((int64_t)L.MPAD * L.MPAD);
  L.r_v = w;  w += large_al(3 * (int64_t)L.KP + 12 * MAXC + 8);
  L.r_total = w;
  return L;
}
struct LargeArgs {
  SmallArgs a;
  double* ws;       // grid * wstride doubles
  int64_t wstride;  // doubles per workspace slot
  double* rec;      // MODE_SETUP / MODE_SOLVEKKT: per-problem records (B x r_total), else NULL
};
// xi: the explicit-inverse build (Li = H^-1 by the sweep, SOCP_F_EXPLICIT_INVERSE);
// gv: the problem's vectors in the HBM workspace instead of LDS (shapes whose
// vectors exceed a CU's 160 KiB of LDS)
const void* large_kernel_ptr(bool xi, bool gv);
const char* large_kernel_name(bool xi, bool gv);

}  // namespace socp
