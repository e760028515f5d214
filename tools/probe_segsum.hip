// Microbenchmark (diagnostic, not product): per-cone segmented sum + broadcast
// over a k=96 vector held as 2 slots x 64 lanes, one wave per SIMD:
//   (a) DPP segmented scan (6 steps) + end-lane LDS exchange
//   (b) ds_add_f64 LDS atomics into per-cone accumulators + read back
// Prints cycles per op (s_memtime) and checks both against a reference sum.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned long long u64;

template <int CTRL, int RM>
__device__ __forceinline__ double dpp(double v) {
  const int lo = __double2loint(v), hi = __double2hiint(v);
  const int l2 = __builtin_amdgcn_update_dpp(0, lo, CTRL, RM, 0xF, false);
  const int h2 = __builtin_amdgcn_update_dpp(0, hi, CTRL, RM, 0xF, false);
  return __hiloint2double(h2, l2);
}
#define WSYNC()                                            \
  do {                                                     \
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront"); \
    __builtin_amdgcn_wave_barrier();                       \
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront"); \
  } while (0)

// cones: [0,32) POC, [32,64) SOC, [64,96) SOC -> cone id per element
__device__ __forceinline__ int cone_of(int i) { return i < 32 ? 0 : (i < 64 ? 1 : 2); }
__device__ __forceinline__ int cone_start(int c) { return 32 * c; }
__device__ __forceinline__ int cone_end(int c) { return 32 * c + 32; }

__global__ void __launch_bounds__(64, 1) probe(const double* in, double* out, u64* cyc, int reps, int mode) {
  __shared__ double part[2][8];
  __shared__ double acc[8];
  const int lane = threadIdx.x;
  double x[2];
  int ci[2], ssl[2], sle[2];
  for (int s = 0; s < 2; ++s) {
    const int i = 64 * s + lane;
    const bool ev = i < 96;
    x[s] = ev ? in[blockIdx.x * 96 + i] : 0.0;
    const int c = ev ? cone_of(i) : 7;
    ci[s] = c;
    const int st = ev ? max(cone_start(c), 64 * s) : i;
    const int en = ev ? min(cone_end(c), 64 * (s + 1)) : i + 1;
    ssl[s] = st - 64 * s;
    sle[s] = en - 1 - 64 * s;
  }
  if (lane < 8) { part[0][lane] = 0; part[1][lane] = 0; acc[lane] = 0; }
  WSYNC();
  double r[2] = {0, 0};
  u64 t0 = __builtin_amdgcn_s_memtime();
  for (int rep = 0; rep < reps; ++rep) {
    if (mode == 0) {
      double v[2] = {x[0] * (1.0 + rep * 1e-9), x[1] * (1.0 + rep * 1e-9)};
      const int rl = lane & 15;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
#define STEP(CTRL, RM, OK)                  \
  {                                         \
    const double y = dpp<CTRL, RM>(v[s]);   \
    v[s] = (OK) ? v[s] + y : v[s];          \
  }
        STEP(0x111, 0xF, rl >= 1 && lane - 1 >= ssl[s])
        STEP(0x112, 0xF, rl >= 2 && lane - 2 >= ssl[s])
        STEP(0x114, 0xF, rl >= 4 && lane - 4 >= ssl[s])
        STEP(0x118, 0xF, rl >= 8 && lane - 8 >= ssl[s])
        STEP(0x142, 0xA, ((lane >> 4) & 1) && ((lane & ~15) - 1 >= ssl[s]))
        STEP(0x143, 0xC, lane >= 32 && 31 >= ssl[s])
#undef STEP
        if (lane == sle[s]) part[s][ci[s]] = v[s];
      }
      WSYNC();
#pragma unroll
      for (int s = 0; s < 2; ++s) r[s] += part[0][ci[s]] + part[1][ci[s]];
      WSYNC();
    } else {
      double v[2] = {x[0] * (1.0 + rep * 1e-9), x[1] * (1.0 + rep * 1e-9)};
#pragma unroll
      for (int s = 0; s < 2; ++s) atomicAdd(&acc[ci[s]], v[s]);
      WSYNC();
      double t[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) t[s] = acc[ci[s]];
      WSYNC();
      if (lane < 8) acc[lane] = 0.0;
      WSYNC();
#pragma unroll
      for (int s = 0; s < 2; ++s) r[s] += t[s];
    }
  }
  u64 t1 = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < 2; ++s) {
    const int i = 64 * s + lane;
    if (i < 96) out[blockIdx.x * 96 + i] = r[s];
  }
  if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int blocks = 1024, reps = 1000;
  std::vector<double> h(blocks * 96);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (double)((i * 2654435761u) % 1000) / 1000.0 - 0.5;
  double *din, *dout;
  u64* dc;
  hipMalloc(&din, h.size() * 8);
  hipMalloc(&dout, h.size() * 8);
  hipMalloc(&dc, blocks * 8);
  hipMemcpy(din, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(probe, dim3(blocks), dim3(64), 0, 0, din, dout, dc, reps, mode);
    hipDeviceSynchronize();
    std::vector<double> o(h.size());
    std::vector<u64> c(blocks);
    hipMemcpy(o.data(), dout, o.size() * 8, hipMemcpyDeviceToHost);
    hipMemcpy(c.data(), dc, blocks * 8, hipMemcpyDeviceToHost);
    double maxerr = 0;
    for (int b = 0; b < blocks; ++b)
      for (int i = 32; i < 96; ++i) {
        double ref = 0;
        int c0 = i < 64 ? 32 : 64;
        for (int j = c0; j < c0 + 32; ++j) ref += h[b * 96 + j];
        double sc = 0;
        for (int rep = 0; rep < reps; ++rep) sc += ref * (1.0 + rep * 1e-9);
        maxerr = fmax(maxerr, fabs(o[b * 96 + i] - sc) / (fabs(sc) + 1));
      }
    double avg = 0;
    for (auto v : c) avg += (double)v;
    avg /= blocks;
    printf("mode %s: %.1f cycles per seg-sum op (1 value x 2 slots), max rel err %.2e\n",
           mode == 0 ? "dpp-scan" : "lds-atomic", avg / reps, maxerr);
  }
  return 0;
}
