// Probe: sustained HBM bandwidth on gfx950 ("verify on the box
// with a copy kernel"): a streaming copy (read + write), a read-only reduction
// and a write-only fill over 4 GiB buffers, 16-byte accesses, grid-stride loops
// with many more workgroups than CUs.  Reports GB/s (bytes moved / kernel time,
// hipEvents, best of 5).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double dbl2 __attribute__((ext_vector_type(2)));

#define CHK(x)                                                                    \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                     \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__global__ void copy_k(const dbl2* __restrict__ a, dbl2* __restrict__ b, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    b[i] = a[i];
}

__global__ void read_k(const dbl2* __restrict__ a, size_t n, double* out) {
  double s = 0.0;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const dbl2 v = a[i];
    s += v.x + v.y;
  }
  if (s == 12345.678) out[0] = s;  // keeps the loads live; never true for the fill value
}

__global__ void fill_k(dbl2* __restrict__ b, size_t n, double v) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    b[i] = (dbl2){v, v};
}

int main() {
  const size_t bytes = (size_t)4 << 30, n = bytes / sizeof(dbl2);
  dbl2 *a, *b;
  double* out;
  CHK(hipMalloc(&a, bytes));
  CHK(hipMalloc(&b, bytes));
  CHK(hipMalloc(&out, 64));
  hipDeviceProp_t prop;
  CHK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(fill_k, dim3(cus * 16), dim3(256), 0, 0, a, n, 1.0);
  CHK(hipDeviceSynchronize());
  printf("device: %s, %d CUs, buffers 2 x %.1f GiB\n", prop.name, cus, bytes / 1073741824.0);
  for (int mult : {8, 16, 32}) {
    const int grid = cus * mult;
    float best_c = 1e30f, best_r = 1e30f, best_f = 1e30f, ms;
    for (int rep = 0; rep < 5; ++rep) {
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(copy_k, dim3(grid), dim3(256), 0, 0, a, b, n);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      CHK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best_c) best_c = ms;
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(read_k, dim3(grid), dim3(256), 0, 0, a, n, out);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      CHK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best_r) best_r = ms;
      CHK(hipEventRecord(e0));
      hipLaunchKernelGGL(fill_k, dim3(grid), dim3(256), 0, 0, b, n, 2.0);
      CHK(hipEventRecord(e1));
      CHK(hipEventSynchronize(e1));
      CHK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best_f) best_f = ms;
    }
    printf("grid %5d x 256: copy %7.1f GB/s (read+write)  read %7.1f GB/s  write %7.1f GB/s\n", grid,
           2.0 * bytes / (best_c * 1e-3) / 1e9, bytes / (best_r * 1e-3) / 1e9, bytes / (best_f * 1e-3) / 1e9);
  }
  CHK(hipFree(a));
  CHK(hipFree(b));
  CHK(hipFree(out));
  return 0;
}
