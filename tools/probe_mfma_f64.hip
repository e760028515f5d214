// Probe: v_mfma_f64_16x16x4_f64 fragment layout + throughput, and v_fma_f64 VALU rate, on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void layout_kernel(const double* A, const double* B, double* D) {
  int l = threadIdx.x;
  // A is 16x4 row-major, B is 4x16 row-major
  double a = A[(l & 15) * 4 + (l >> 4)];
  double b = B[(l >> 4) * 16 + (l & 15)];
  d4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) {
    int row = (l >> 4) + 4 * r, col = l & 15;
    D[row * 16 + col] = c[r];
  }
}

template <int NACC>
__global__ void mfma_rate(double* out, int iters, double seed) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = (d4){0, 0, 0, 0};
  double a = seed + threadIdx.x * 1e-3, b = seed * 0.5 - threadIdx.x * 1e-3;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int NCH>
__global__ void fma_rate(double* out, int iters, double seed) {
  double x[NCH];
  for (int i = 0; i < NCH; ++i) x[i] = seed + i + threadIdx.x;
  double m = 0.999999, a = 1e-7;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NCH; ++i) x[i] = fma(x[i], m, a);
  }
  double s = 0;
  for (int i = 0; i < NCH; ++i) s += x[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  double hA[64], hB[64], hD[256], ref[256];
  for (int i = 0; i < 64; ++i) { hA[i] = (i * 7) % 13 - 6; hB[i] = (i * 5) % 11 - 5 + 0.5 * (i % 3); }
  for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) { double s = 0; for (int k = 0; k < 4; ++k) s += hA[i*4+k] * hB[k*16+j]; ref[i*16+j] = s; }
  double *dA, *dB, *dD, *dout;
  hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dD, 2048);
  hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
  layout_kernel<<<1, 64>>>(dA, dB, dD);
  hipMemcpy(hD, dD, 2048, hipMemcpyDeviceToHost);
  int bad = 0; for (int i = 0; i < 256; ++i) if (hD[i] != ref[i]) ++bad;
  printf("layout check: %d mismatches of 256\n", bad);

  int nblk = 256 * 4, nthr = 64, iters = 4096;
  hipMalloc(&dout, nblk * nthr * 8 * 4);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  float ms;
#define RUN(K, NAME, FLOP_PER)                                                      \
  K<<<nblk, nthr>>>(dout, 16, 1.0); hipDeviceSynchronize();                         \
  hipEventRecord(e0); K<<<nblk, nthr>>>(dout, iters, 1.0); hipEventRecord(e1);      \
  hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);                        \
  printf("%-28s blocks=%d : %.3f ms  %.2f TFLOP/s\n", NAME, nblk, ms,               \
         (double)nblk * iters * (FLOP_PER) / (ms * 1e-3) / 1e12);
  RUN(mfma_rate<1>, "mfma_f64 16x16x4 acc=1", 1 * 2048.0)
  RUN(mfma_rate<2>, "mfma_f64 16x16x4 acc=2", 2 * 2048.0)
  RUN(mfma_rate<4>, "mfma_f64 16x16x4 acc=4", 4 * 2048.0)
  RUN(mfma_rate<8>, "mfma_f64 16x16x4 acc=8", 8 * 2048.0)
  RUN(fma_rate<4>, "v_fma_f64 chains=4", 4 * 64 * 2.0)
  RUN(fma_rate<8>, "v_fma_f64 chains=8", 8 * 64 * 2.0)
  RUN(fma_rate<16>, "v_fma_f64 chains=16", 16 * 64 * 2.0)
  nblk = 256 * 8;
  RUN(mfma_rate<4>, "mfma_f64 acc=4 (8 wv/CU)", 4 * 2048.0)
  RUN(fma_rate<8>, "v_fma_f64 ch=8 (8 wv/CU)", 8 * 64 * 2.0)
  // single wave latency: 1 block
  nblk = 1;
  RUN(mfma_rate<1>, "mfma dep chain 1 wave", 2048.0)
  printf("  -> cycles per dependent mfma @2.4GHz: %.1f\n", ms * 1e-3 * 2.4e9 / iters);
  RUN(mfma_rate<4>, "mfma 4acc 1 wave", 4 * 2048.0)
  printf("  -> cycles per mfma (4 indep) @2.4GHz: %.1f\n", ms * 1e-3 * 2.4e9 / iters / 4);
  RUN(fma_rate<1>, "fma dep chain 1 wave", 64 * 2.0)
  printf("  -> cycles per dependent fma @2.4GHz: %.1f\n", ms * 1e-3 * 2.4e9 / iters);
  RUN(fma_rate<16>, "fma 16 chains 1 wave", 16 * 64 * 2.0)
  printf("  -> cycles per fma (16 indep) @2.4GHz: %.1f\n", ms * 1e-3 * 2.4e9 / iters / 16);
  return 0;
}
