// Probe: variants of the 16x16 tile factorisation (socp_small.hpp factor_tile)
// on one wave per SIMD, s_memtime cycles per factorisation, each trip's input
// depending on the last (as tools/probe_tile.hip):
//   cur   : factor_tile as the register kernel runs it
//   defer : the identity tile's rank-4 update of block B issued inside block
//           B+1's pivot chain (after its first rsq) instead of behind block B
//   donly : the D updates only (no inverse rows): what the W half costs
// Prints the max |difference| of W between cur and defer (must be 0: the same
// operations on the same values).
#include "../socp.jl_amd/csrc/socp_small.hpp"
#include <cstdio>
using namespace socp;
typedef unsigned long long u64;

template <int B, bool DEFER, bool WROWS>
__device__ __forceinline__ void tb(d4& Dt, d4& It, d4& W, bool& ok, double pR, double pW) {
  if constexpr (B < 4) {
    LANE_IDS();
    const double v = Dt[B];
    const double a00 = readlane_d(v, 4 * B), a01 = readlane_d(v, 4 * B + 1), a02 = readlane_d(v, 4 * B + 2),
                 a03 = readlane_d(v, 4 * B + 3);
    const double a11 = readlane_d(v, 16 + 4 * B + 1), a12 = readlane_d(v, 16 + 4 * B + 2),
                 a13 = readlane_d(v, 16 + 4 * B + 3);
    const double a22 = readlane_d(v, 32 + 4 * B + 2), a23 = readlane_d(v, 32 + 4 * B + 3);
    const double a33 = readlane_d(v, 48 + 4 * B + 3);
    const double rs0 = rsqrt_tile(a00);
    if constexpr (DEFER && WROWS && B > 0) It = __builtin_amdgcn_mfma_f64_16x16x4f64(pR, pW, It, 0, 0, 1);
    const double r01 = a01 * rs0, r02 = a02 * rs0, r03 = a03 * rs0;
    const double s11 = fma(-r01, r01, a11);
    const double rs1 = rsqrt_tile(s11);
    const double r12 = fma(-r01, r02, a12) * rs1, r13 = fma(-r01, r03, a13) * rs1;
    const double s22 = fma(-r12, r12, fma(-r02, r02, a22));
    const double rs2 = rsqrt_tile(s22);
    const double r23 = fma(-r12, r13, fma(-r02, r03, a23)) * rs2;
    const double s33 = fma(-r23, r23, fma(-r13, r13, fma(-r03, r03, a33)));
    const double rs3 = rsqrt_tile(s33);
    ok = ok && (a00 > 0.0) && (s11 > 0.0) && (s22 > 0.0) && (s33 > 0.0);
    double V[4];
    row_bcast4(v, V);
    const double R0 = V[0] * rs0;
    const double R1 = fma(-r01, R0, V[1]) * rs1;
    const double R2 = fma(-r12, R1, fma(-r02, R0, V[2])) * rs2;
    const double R3 = fma(-r23, R2, fma(-r13, R1, fma(-r03, R0, V[3]))) * rs3;
    const double R = g == 0 ? R0 : (g == 1 ? R1 : (g == 2 ? R2 : R3));
    double Wb = 0.0;
    if constexpr (WROWS) {
      double X[4];
      row_bcast4(It[B], X);
      const double W0 = X[0] * rs0;
      const double W1 = fma(-r01, W0, X[1]) * rs1;
      const double W2 = fma(-r12, W1, fma(-r02, W0, X[2])) * rs2;
      const double W3 = fma(-r23, W2, fma(-r13, W1, fma(-r03, W0, X[3]))) * rs3;
      Wb = g == 0 ? W0 : (g == 1 ? W1 : (g == 2 ? W2 : W3));
      W[B] = Wb;
    } else {
      W[B] = R;
    }
    if constexpr (B < 3) {
      Dt = __builtin_amdgcn_mfma_f64_16x16x4f64(R, R, Dt, 0, 0, 1);
      if constexpr (!DEFER && WROWS) It = __builtin_amdgcn_mfma_f64_16x16x4f64(R, Wb, It, 0, 0, 1);
    }
    tb<B + 1, DEFER, WROWS>(Dt, It, W, ok, R, Wb);
  }
}
template <bool DEFER, bool WROWS>
__device__ __forceinline__ void ftile(d4 Dt, d4& W, bool& ok) {
  LANE_IDS();
  d4 It;
#pragma unroll
  for (int r = 0; r < 4; ++r) It[r] = (g + 4 * r == cl) ? 1.0 : 0.0;
  W = It;
  tb<0, DEFER, WROWS>(Dt, It, W, ok, 0.0, 0.0);
}

template <int MODE>
__global__ void __launch_bounds__(64, 1) probe(double* out, u64* cyc, int iters, double seed) {
  const int l = threadIdx.x, g = l >> 4, cl = l & 15;
  d4 D;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = g + 4 * r, j = cl;
    D[r] = (i == j ? 20.0 : 0.0) + 1.0 / (1.0 + i + j) + seed * 1e-3;
  }
  d4 W = D;
  bool ok = true;
  const u64 t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) factor_tile(D, W, ok);
    if (MODE == 1) ftile<false, true>(D, W, ok);
    if (MODE == 2) ftile<true, true>(D, W, ok);
    if (MODE == 3) ftile<false, false>(D, W, ok);
#pragma unroll
    for (int r = 0; r < 4; ++r) D[r] = fma(W[r], 1e-300, D[r]);
  }
  const u64 t1 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int r = 0; r < 4; ++r) out[(blockIdx.x * 64 + l) * 4 + r] = W[r] + (ok ? 0.0 : 1.0);
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
static double run(const char* name, double* dout, u64* dc, int blocks, int iters, double* hw) {
  hipLaunchKernelGGL((probe<MODE>), dim3(blocks), dim3(64), 0, 0, dout, dc, iters, 1.0);
  hipDeviceSynchronize();
  hipLaunchKernelGGL((probe<MODE>), dim3(blocks), dim3(64), 0, 0, dout, dc, iters, 1.0);
  hipDeviceSynchronize();
  u64* h = new u64[blocks];
  hipMemcpy(h, dc, sizeof(u64) * blocks, hipMemcpyDeviceToHost);
  hipMemcpy(hw, dout, sizeof(double) * blocks * 256, hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < blocks; ++i) avg += (double)h[i];
  avg /= blocks;
  delete[] h;
  printf("%-10s %9.1f cycles per factorisation\n", name, avg / iters);
  return avg / iters;
}

int main() {
  const int blocks = 1024, iters = 256;
  double* dout;
  u64* dc;
  hipMalloc(&dout, sizeof(double) * blocks * 256);
  hipMalloc(&dc, sizeof(u64) * blocks);
  double* w0 = new double[blocks * 256];
  double* w1 = new double[blocks * 256];
  double* w2 = new double[blocks * 256];
  run<0>("kernel", dout, dc, blocks, iters, w0);
  run<1>("cur", dout, dc, blocks, iters, w1);
  run<2>("defer", dout, dc, blocks, iters, w2);
  run<3>("donly", dout, dc, blocks, iters, w0);
  double md = 0;
  for (int i = 0; i < blocks * 256; ++i) md = fmax(md, fabs(w1[i] - w2[i]));
  printf("max |W(cur) - W(defer)| = %g\n", md);
  return 0;
}
