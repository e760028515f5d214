// Probe: can one wave's f64 VALU work proceed while its own f64 MFMAs run?
// One wave per SIMD (1024 one-wave blocks); s_memtime cycles per loop trip.
//   mfma   : 4 independent v_mfma_f64_16x16x4_f64 chains
//   fma    : 16 independent v_fma_f64 chains (F per trip)
//   mix    : both in the same loop body
//   mix_i  : MFMAs + integer VALU (v_add_u32), mix_l: MFMAs + LDS reads
// If mix ~ max(mfma, fma) the pipes overlap; if ~ sum they share the datapath.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64;

template <int MODE, int NF>
__global__ void __launch_bounds__(64, 1) probe(double* out, u64* cyc, u64* rt, int iters, double seed) {
  __shared__ double lds[256];
  const int l = threadIdx.x;
  lds[l] = seed + l;
  lds[l + 64] = seed - l;
  __syncthreads();
  double a = seed + l * 1e-3, b = seed - l * 1e-3;
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double f[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) f[i] = seed * (i + 1) + l;
  unsigned iv[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) iv[i] = l + i;
  double ls = 0.0;
  const u64 r0 = __builtin_amdgcn_s_memrealtime();
  const u64 t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0 || MODE == 2 || MODE == 3 || MODE == 4) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
    }
    if (MODE == 1 || MODE == 2) {
#pragma unroll
      for (int k = 0; k < NF; ++k) f[k % 16] = fma(f[k % 16], 0.999999, 1e-9);
    }
    if (MODE == 3) {
#pragma unroll
      for (int k = 0; k < NF; ++k) iv[k % 16] = iv[k % 16] * 3u + 7u;
    }
    if (MODE == 4) {
#pragma unroll
      for (int k = 0; k < NF; ++k) ls += lds[(l + k * 5 + it) & 127];
    }
  }
  const u64 t1 = __builtin_amdgcn_s_memtime();
  const u64 r1 = __builtin_amdgcn_s_memrealtime();
  double acc = c0[0] + c1[1] + c2[2] + c3[3] + ls;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc += f[i] + (double)iv[i];
  out[blockIdx.x * 64 + l] = acc;
  if (l == 0) { cyc[blockIdx.x] = t1 - t0; rt[blockIdx.x] = r1 - r0; }
}

template <int MODE, int NF>
static double run(const char* name, double* dout, u64* dc, int blocks, int iters) {
  static u64* drt = nullptr;
  if (!drt) hipMalloc(&drt, sizeof(u64) * 4096);
  hipLaunchKernelGGL((probe<MODE, NF>), dim3(blocks), dim3(64), 0, 0, dout, dc, drt, iters, 1.0);
  hipDeviceSynchronize();
  hipLaunchKernelGGL((probe<MODE, NF>), dim3(blocks), dim3(64), 0, 0, dout, dc, drt, iters, 1.0);
  hipDeviceSynchronize();
  u64* h = new u64[blocks];
  u64* r = new u64[blocks];
  hipMemcpy(h, dc, sizeof(u64) * blocks, hipMemcpyDeviceToHost);
  hipMemcpy(r, drt, sizeof(u64) * blocks, hipMemcpyDeviceToHost);
  double avg = 0, art = 0;
  for (int i = 0; i < blocks; ++i) { avg += (double)h[i]; art += (double)r[i]; }
  avg /= blocks;
  art /= blocks;
  delete[] h;
  delete[] r;
  // s_memrealtime ticks at 100 MHz: memtime ticks per ns and ns per trip
  printf("%-28s blocks %4d %8.1f memtime/trip %7.1f ns/trip (memtime %.2f GHz)\n", name, blocks, avg / iters,
         art * 10.0 / iters, avg / (art * 10.0));
  return avg / iters;
}

int main() {
  const int blocks = 1024, iters = 4096;
  double* dout;
  u64* dc;
  hipMalloc(&dout, sizeof(double) * blocks * 64);
  hipMalloc(&dc, sizeof(u64) * blocks);
  run<0, 16>("mfma x4 (one CU)", dout, dc, 4, iters);
  run<1, 16>("fma64 x16 (one CU)", dout, dc, 4, iters);
  run<2, 16>("mfma x4 + fma64 x16 (1 CU)", dout, dc, 4, iters);
  run<0, 16>("mfma x4", dout, dc, blocks, iters);
  run<1, 16>("fma64 x16", dout, dc, blocks, iters);
  run<1, 32>("fma64 x32", dout, dc, blocks, iters);
  run<2, 16>("mfma x4 + fma64 x16", dout, dc, blocks, iters);
  run<2, 32>("mfma x4 + fma64 x32", dout, dc, blocks, iters);
  run<2, 64>("mfma x4 + fma64 x64", dout, dc, blocks, iters);
  run<3, 32>("mfma x4 + u32 x32", dout, dc, blocks, iters);
  run<3, 64>("mfma x4 + u32 x64", dout, dc, blocks, iters);
  run<4, 8>("mfma x4 + lds x8", dout, dc, blocks, iters);
  return 0;
}
