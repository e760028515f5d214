// Probe: what one 16x16 tile factorisation (socp_small.hpp factor_tile, the
// register kernel's Cholesky / inverse building block) costs one wave, and
// the dependent latencies of the instructions on its chain.  One wave per
// SIMD (1024 one-wave blocks), s_memtime cycles per loop trip.
//   fma_chain   : dependent v_fma_f64
//   rsq_chain   : dependent v_rsq_f64
//   rsqnr_chain : dependent rsqrt_tile (rsq + one Newton step)
//   rl_chain    : v_readlane -> f64 op -> next readlane (SGPR round trip)
//   mfma_chain  : dependent v_mfma_f64_16x16x4_f64 accumulations
//   factor_tile : the tile factorisation, each trip's input depending on the last
#include "../socp.jl_amd/csrc/socp_small.hpp"
#include <cstdio>
using namespace socp;
typedef unsigned long long u64;

template <int MODE>
__global__ void __launch_bounds__(64, 1) probe(double* out, u64* cyc, int iters, double seed) {
  const int l = threadIdx.x, g = l >> 4, cl = l & 15;
  double x = seed + l * 1e-3;
  d4 D;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = g + 4 * r, j = cl;
    D[r] = (i == j ? 20.0 : 0.0) + 1.0 / (1.0 + i + j) + seed * 1e-3;
  }
  d4 W = D, C = {0, 0, 0, 0};
  bool ok = true;
  const u64 t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) {
#pragma unroll
      for (int k = 0; k < 32; ++k) x = fma(x, 0.999999, 1e-9);
    } else if (MODE == 1) {
#pragma unroll
      for (int k = 0; k < 32; ++k) x = __builtin_amdgcn_rsq(x) + 1.0;
    } else if (MODE == 2) {
#pragma unroll
      for (int k = 0; k < 32; ++k) x = rsqrt_tile(x) + 1.0;
    } else if (MODE == 3) {
#pragma unroll
      for (int k = 0; k < 32; ++k) x = readlane_d(x, k & 63) * 0.999 + 1e-9;
    } else if (MODE == 4) {
#pragma unroll
      for (int k = 0; k < 32; ++k) C = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, C, 0, 0, 0);
    } else if (MODE == 5) {
      factor_tile(D, W, ok);
#pragma unroll
      for (int r = 0; r < 4; ++r) D[r] = fma(W[r], 1e-300, D[r]);
    }
  }
  const u64 t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + l] = x + C[0] + W[0] + W[1] + W[2] + W[3] + (ok ? 0.0 : 1.0);
  if (l == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
static void run(const char* name, double per, double* dout, u64* dc, int blocks, int iters) {
  hipLaunchKernelGGL((probe<MODE>), dim3(blocks), dim3(64), 0, 0, dout, dc, iters, 1.0);
  hipDeviceSynchronize();
  hipLaunchKernelGGL((probe<MODE>), dim3(blocks), dim3(64), 0, 0, dout, dc, iters, 1.0);
  hipDeviceSynchronize();
  u64* h = new u64[blocks];
  hipMemcpy(h, dc, sizeof(u64) * blocks, hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < blocks; ++i) avg += (double)h[i];
  avg /= blocks;
  delete[] h;
  printf("%-14s %9.1f cycles/trip  %7.1f cycles/op\n", name, avg / iters, avg / iters / per);
}

int main() {
  const int blocks = 1024, iters = 2048;
  double* dout;
  u64* dc;
  hipMalloc(&dout, sizeof(double) * blocks * 64);
  hipMalloc(&dc, sizeof(u64) * blocks);
  run<0>("fma_chain", 32, dout, dc, blocks, iters);
  run<1>("rsq_chain", 32, dout, dc, blocks, iters);
  run<2>("rsqnr_chain", 32, dout, dc, blocks, iters);
  run<3>("rl_chain", 32, dout, dc, blocks, iters);
  run<4>("mfma_chain", 32, dout, dc, blocks, iters);
  run<5>("factor_tile", 1, dout, dc, blocks, iters / 8);
  return 0;
}
