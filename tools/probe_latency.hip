// Microbenchmark (diagnostic, not product): dependent-chain latencies on gfx950
// at one wave per SIMD (1024 one-wave blocks), in s_memtime cycles per op.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned long long u64;
#define N 256

template <int MODE>
__global__ void __launch_bounds__(64, 1) lat(double* out, u64* cyc, double seed) {
  __shared__ double sh[128];
  const int lane = threadIdx.x;
  double x = seed + lane * 1e-3, y = 1.0000001, z = 0.999999;
  sh[lane] = x;
  sh[64 + lane] = y;
  __builtin_amdgcn_s_waitcnt(0);
  u64 t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
  for (int i = 0; i < N; ++i) {
    if (MODE == 0) x = fma(x, y, z);                       // dependent v_fma_f64
    if (MODE == 1) x = x * y;                              // dependent v_mul_f64
    if (MODE == 2) x = __builtin_amdgcn_rcp(x);           // dependent v_rcp_f64
    if (MODE == 3) {                                       // dependent 2x DPP mov (64-bit) + add
      const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), 0x111, 0xF, 0xF, false);
      const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), 0x111, 0xF, 0xF, false);
      x = x + __hiloint2double(hi, lo) * 1e-3;
    }
    if (MODE == 4) {                                       // dependent LDS write -> read
      sh[lane] = x;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      x = sh[(lane + 1) & 63] + 1e-9;
    }
    if (MODE == 5) {                                       // dependent readlane (SGPR) + VALU
      const int lo = __builtin_amdgcn_readlane(__double2loint(x), 5);
      const int hi = __builtin_amdgcn_readlane(__double2hiint(x), 5);
      x = __hiloint2double(hi, lo) * y;
    }
    if (MODE == 6) {                                       // 8 independent fma chains (throughput)
      x = fma(x, y, z);
      y = fma(y, z, x);
    }
    if (MODE == 7) x = sqrt(x) + 1.0;                      // dependent IEEE sqrt (library sequence)
    if (MODE == 8) x = 1.0 / x + 0.5;                      // dependent IEEE divide
  }
  __builtin_amdgcn_s_waitcnt(0);
  u64 t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + lane] = x + y;
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
void run(const char* name, double* dout, u64* dc, int blocks) {
  hipLaunchKernelGGL(lat<MODE>, dim3(blocks), dim3(64), 0, 0, dout, dc, 1.5);
  hipLaunchKernelGGL(lat<MODE>, dim3(blocks), dim3(64), 0, 0, dout, dc, 1.5);
  (void)hipDeviceSynchronize();
  std::vector<u64> c(blocks);
  (void)hipMemcpy(c.data(), dc, blocks * 8, hipMemcpyDeviceToHost);
  double avg = 0;
  for (auto v : c) avg += (double)v;
  printf("%-40s %7.1f cycles/op (blocks=%d)\n", name, avg / blocks / N, blocks);
}

int main() {
  double* dout;
  u64* dc;
  (void)hipMalloc(&dout, 4096 * 64 * 8);
  (void)hipMalloc(&dc, 4096 * 8);
  for (int blocks : {1024, 4096}) {
    run<0>("v_fma_f64 dependent", dout, dc, blocks);
    run<1>("v_mul_f64 dependent", dout, dc, blocks);
    run<2>("v_rcp_f64 dependent", dout, dc, blocks);
    run<3>("dpp row_shr (2x b32) + fma dependent", dout, dc, blocks);
    run<4>("ds_write+ds_read dependent", dout, dc, blocks);
    run<5>("readlane x2 + mul dependent", dout, dc, blocks);
    run<6>("2 interleaved fma chains (per 2 ops)", dout, dc, blocks);
    run<7>("sqrt (IEEE) + add dependent", dout, dc, blocks);
    run<8>("1/x (IEEE) + add dependent", dout, dc, blocks);
  }
  return 0;
}
