// Probe: do two waves on ONE SIMD overlap f64 MFMA with f64 VALU?
// One 512-thread workgroup per CU (8 waves, two per SIMD).  Wave w's SIMD is
// read from HW_ID and recorded, so the pairing is checked, not assumed.
// Modes (per-wave role chosen from the wave index w = tid / 64):
//   0 "mfma lo"     : waves 0-3 run 4 independent v_mfma_f64_16x16x4 chains, 4-7 exit
//   1 "fma lo"      : waves 0-3 run NF independent v_fma_f64, 4-7 exit
//   2 "mfma|fma"    : waves 0-3 MFMA, waves 4-7 FMA       (cross-wave overlap?)
//   3 "mix lo"      : waves 0-3 run MFMA + NF FMA in one stream, 4-7 exit
//   4 "mix all"     : all 8 waves run the mixed stream     (2 mixed waves per SIMD)
//   5 "mfma all"    : all 8 waves MFMA
//   6 "lds-chain lo": waves 0-3: MFMA + a dependent LDS read chain (latency-bound)
//   7 "lds-chain all": all 8 waves: MFMA + dependent LDS chain
// Reported: s_memtime cycles per loop trip, averaged over the active waves.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64;

template <int MODE, int NF>
__global__ void __launch_bounds__(512, 1) probe2(double* out, u64* cyc, int* simd, int iters, double seed) {
  __shared__ double lds[512];
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  lds[t] = (double)((t * 7 + 3) & 511);
  __syncthreads();
  const bool lo = w < 4;
  bool do_m = false, do_f = false, do_l = false;
  if (MODE == 0) do_m = lo;
  if (MODE == 1) do_f = lo;
  if (MODE == 2) { do_m = lo; do_f = !lo; }
  if (MODE == 3) { do_m = lo; do_f = lo; }
  if (MODE == 4) { do_m = true; do_f = true; }
  if (MODE == 5) do_m = true;
  if (MODE == 6) { do_m = lo; do_l = lo; }
  if (MODE == 7) { do_m = true; do_l = true; }
  const unsigned hwid = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_REG_HW_ID, all 32 bits
  if (l == 0) simd[blockIdx.x * 8 + w] = (hwid >> 4) & 3;
  if (!(do_m || do_f || do_l)) return;
  double a = seed + l * 1e-3, b = seed - l * 1e-3;
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double f[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) f[i] = seed * (i + 1) + l;
  int li = l;
  double ls = 0;
  const u64 t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (do_m) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
    }
    if (do_f) {
#pragma unroll
      for (int k = 0; k < NF; ++k) f[k % 16] = fma(f[k % 16], 0.999999, 1e-9);
    }
    if (do_l) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const double v = lds[li];
        li = ((int)v + k) & 511;
        ls += v;
      }
    }
  }
  const u64 t1 = __builtin_amdgcn_s_memtime();
  double acc = c0[0] + c1[1] + c2[2] + c3[3] + ls;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc += f[i];
  out[blockIdx.x * 512 + t] = acc;
  if (l == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
}

template <int MODE, int NF>
static void run(const char* name, double* dout, u64* dc, int* ds, int blocks, int iters) {
  hipMemset(dc, 0, sizeof(u64) * blocks * 8);
  hipLaunchKernelGGL((probe2<MODE, NF>), dim3(blocks), dim3(512), 0, 0, dout, dc, ds, iters, 1.0);
  hipDeviceSynchronize();
  hipMemset(dc, 0, sizeof(u64) * blocks * 8);
  hipLaunchKernelGGL((probe2<MODE, NF>), dim3(blocks), dim3(512), 0, 0, dout, dc, ds, iters, 1.0);
  hipDeviceSynchronize();
  u64* h = new u64[blocks * 8];
  int* s = new int[blocks * 8];
  hipMemcpy(h, dc, sizeof(u64) * blocks * 8, hipMemcpyDeviceToHost);
  hipMemcpy(s, ds, sizeof(int) * blocks * 8, hipMemcpyDeviceToHost);
  double alo = 0, ahi = 0;
  int nlo = 0, nhi = 0, pair_ok = 0;
  for (int b = 0; b < blocks; ++b) {
    for (int w = 0; w < 8; ++w) {
      if (!h[b * 8 + w]) continue;
      if (w < 4) { alo += (double)h[b * 8 + w]; ++nlo; } else { ahi += (double)h[b * 8 + w]; ++nhi; }
    }
    int ok = 1;
    for (int w = 0; w < 4; ++w) ok &= (s[b * 8 + w] == s[b * 8 + w + 4]);
    pair_ok += ok;
  }
  printf("%-34s waves0-3 %8.1f cyc/trip  waves4-7 %8.1f cyc/trip  (w and w+4 on one SIMD in %d/%d blocks; simd of w0..7 in block 0: %d%d%d%d%d%d%d%d)\n",
         name, nlo ? alo / nlo / iters : 0.0, nhi ? ahi / nhi / iters : 0.0, pair_ok, blocks,
         s[0], s[1], s[2], s[3], s[4], s[5], s[6], s[7]);
  delete[] h;
  delete[] s;
}

int main() {
  const int blocks = 256, iters = 4096;
  double* dout;
  u64* dc;
  int* ds;
  hipMalloc(&dout, sizeof(double) * blocks * 512);
  hipMalloc(&dc, sizeof(u64) * blocks * 8);
  hipMalloc(&ds, sizeof(int) * blocks * 8);
  run<0, 16>("mfma x4 (1 wave/SIMD)", dout, dc, ds, blocks, iters);
  run<1, 16>("fma64 x16 (1 wave/SIMD)", dout, dc, ds, blocks, iters);
  run<1, 64>("fma64 x64 (1 wave/SIMD)", dout, dc, ds, blocks, iters);
  run<2, 16>("mfma | fma64 x16 (2 waves/SIMD)", dout, dc, ds, blocks, iters);
  run<2, 64>("mfma | fma64 x64 (2 waves/SIMD)", dout, dc, ds, blocks, iters);
  run<3, 16>("mix x16 (1 wave/SIMD)", dout, dc, ds, blocks, iters);
  run<4, 16>("mix x16 (2 waves/SIMD)", dout, dc, ds, blocks, iters);
  run<3, 32>("mix x32 (1 wave/SIMD)", dout, dc, ds, blocks, iters);
  run<4, 32>("mix x32 (2 waves/SIMD)", dout, dc, ds, blocks, iters);
  run<5, 16>("mfma x4 (2 waves/SIMD)", dout, dc, ds, blocks, iters);
  run<6, 16>("mfma + lds chain (1 wave/SIMD)", dout, dc, ds, blocks, iters);
  run<7, 16>("mfma + lds chain (2 waves/SIMD)", dout, dc, ds, blocks, iters);
  return 0;
}
