// Probe: what does a second wave per SIMD buy for a C2-like f64 instruction mix?
// One 512-thread workgroup per CU (8 waves, two per SIMD; wave w's SIMD is
// read from HW_ID, so the w / w+4 pairing is checked, not assumed).  Each
// active wave runs `iters` trips of a stream; the figure of merit is the
// SPAN of the whole block (max end - min start over its waves, s_memtime),
// divided by the trips ALL active waves ran: shader cycles per trip of
// SIMD throughput.  A wave's own cycles/trip are printed too, but under
// age-priority arbitration the younger wave runs mostly after the older one,
// so only the span says what co-residence buys.
// Streams (per trip):
//   M  : 4 independent v_mfma_f64_16x16x4 chains
//   F  : NF independent v_fma_f64 (16 chains)
//   I  : NF 32-bit integer VALU ops (v_mad_u32-like)
//   L  : a dependent chain of 4 LDS reads (address from the previous value)
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64;

template <bool M, int NF, int NI, bool LC, bool ALL>
__global__ void __launch_bounds__(512, 1) probe2(double* out, u64* t0s, u64* t1s, int* simd, int iters, double seed) {
  __shared__ double lds[512];
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  lds[t] = (double)((t * 7 + 3) & 511);
  __syncthreads();
  const unsigned hwid = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_REG_HW_ID
  if (l == 0) simd[blockIdx.x * 8 + w] = (hwid >> 4) & 3;
  if (!ALL && w >= 4) return;
  double a = seed + l * 1e-3, b = seed - l * 1e-3;
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double f[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) f[i] = seed * (i + 1) + l;
  unsigned iv[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) iv[i] = l + i;
  int li = l;
  double ls = 0;
  const u64 t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (M) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < NF; ++k) f[k % 16] = fma(f[k % 16], 0.999999, 1e-9);
#pragma unroll
    for (int k = 0; k < NI; ++k) iv[k % 16] = iv[k % 16] * 3u + 7u;
    if (LC) {
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
  for (int i = 0; i < 16; ++i) acc += f[i] + (double)iv[i];
  out[blockIdx.x * 512 + t] = acc;
  if (l == 0) {
    t0s[blockIdx.x * 8 + w] = t0;
    t1s[blockIdx.x * 8 + w] = t1;
  }
}

template <bool M, int NF, int NI, bool LC, bool ALL>
static double run(const char* name, double* dout, u64* d0, u64* d1, int* ds, int blocks, int iters) {
  for (int rep = 0; rep < 2; ++rep) {
    hipMemset(d0, 0, sizeof(u64) * blocks * 8);
    hipMemset(d1, 0, sizeof(u64) * blocks * 8);
    hipLaunchKernelGGL((probe2<M, NF, NI, LC, ALL>), dim3(blocks), dim3(512), 0, 0, dout, d0, d1, ds, iters, 1.0);
    hipDeviceSynchronize();
  }
  u64* h0 = new u64[blocks * 8];
  u64* h1 = new u64[blocks * 8];
  int* s = new int[blocks * 8];
  hipMemcpy(h0, d0, sizeof(u64) * blocks * 8, hipMemcpyDeviceToHost);
  hipMemcpy(h1, d1, sizeof(u64) * blocks * 8, hipMemcpyDeviceToHost);
  hipMemcpy(s, ds, sizeof(int) * blocks * 8, hipMemcpyDeviceToHost);
  const int nw = ALL ? 8 : 4;
  double span = 0, own_lo = 0, own_hi = 0;
  int pair_ok = 0;
  for (int b = 0; b < blocks; ++b) {
    u64 mn = ~0ull, mx = 0;
    for (int w = 0; w < nw; ++w) {
      mn = h0[b * 8 + w] < mn ? h0[b * 8 + w] : mn;
      mx = h1[b * 8 + w] > mx ? h1[b * 8 + w] : mx;
      (w < 4 ? own_lo : own_hi) += (double)(h1[b * 8 + w] - h0[b * 8 + w]);
    }
    span += (double)(mx - mn);
    int ok = 1;
    for (int w = 0; w < 4; ++w) ok &= (s[b * 8 + w] == s[b * 8 + w + 4]);
    pair_ok += ok;
  }
  // per SIMD: (waves per SIMD) x iters trips in the span
  const double per_trip = span / blocks / ((nw / 4) * (double)iters);
  printf("%-40s span/trip %7.1f cyc   own: w0-3 %7.1f  w4-7 %7.1f cyc/trip   (pairs on one SIMD %d/%d)\n", name,
         per_trip, own_lo / (4.0 * blocks * iters), ALL ? own_hi / (4.0 * blocks * iters) : 0.0, pair_ok, blocks);
  delete[] h0;
  delete[] h1;
  delete[] s;
  return per_trip;
}

int main() {
  const int blocks = 256, iters = 2048;
  double* dout;
  u64 *d0, *d1;
  int* ds;
  hipMalloc(&dout, sizeof(double) * blocks * 512);
  hipMalloc(&d0, sizeof(u64) * blocks * 8);
  hipMalloc(&d1, sizeof(u64) * blocks * 8);
  hipMalloc(&ds, sizeof(int) * blocks * 8);
#define PAIR(NAME, M, NF, NI, LC)                                                              \
  {                                                                                            \
    const double one = run<M, NF, NI, LC, false>(NAME " (1 wave/SIMD)", dout, d0, d1, ds, blocks, iters); \
    const double two = run<M, NF, NI, LC, true>(NAME " (2 waves/SIMD)", dout, d0, d1, ds, blocks, iters); \
    printf("%-40s -> throughput gain of the second wave: %.2fx\n", NAME, one / two);          \
  }
  PAIR("mfma x4", true, 0, 0, false)
  PAIR("fma64 x32", false, 32, 0, false)
  PAIR("u32 x32", false, 0, 32, false)
  PAIR("lds chain x4", false, 0, 0, true)
  PAIR("mfma x4 + fma64 x16", true, 16, 0, false)
  PAIR("mfma x4 + fma64 x32", true, 32, 0, false)
  PAIR("mfma x4 + u32 x32", true, 0, 32, false)
  PAIR("mfma x4 + lds chain", true, 0, 0, true)
  PAIR("mfma x4 + fma64 x32 + u32 x32 + lds", true, 32, 32, true)
  PAIR("mfma x4 + fma64 x48 + u32 x24 + lds", true, 48, 24, true)
  return 0;
}
