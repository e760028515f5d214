// Probe: accuracy of v_rcp_f64 and of one / two Newton steps against the IEEE
// quotient 1.0/d, in ulps, over 2^24 values of d spread over [1e-8, 1e8].
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>

__global__ void rcp_k(int n, unsigned long long* worst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double t = (double)i / n;
  const double d = exp2(-26.6 + 53.2 * t) * (1.0 + 0.37 * sin(1e4 * t));
  const double q = 1.0 / d;
  double r = __builtin_amdgcn_rcp(d);
  double e = fma(-d, r, 1.0);
  const double r1 = fma(r, e, r);
  e = fma(-d, r1, 1.0);
  const double r2 = fma(r1, e, r1);
  const long long qb = __double_as_longlong(q);
  const unsigned long long u0 = llabs(__double_as_longlong(r) - qb), u1 = llabs(__double_as_longlong(r1) - qb),
                           u2 = llabs(__double_as_longlong(r2) - qb);
  atomicMax(worst + 0, u0);
  atomicMax(worst + 1, u1);
  atomicMax(worst + 2, u2);
}

int main() {
  unsigned long long* w;
  hipMalloc(&w, 3 * sizeof(unsigned long long));
  hipMemset(w, 0, 3 * sizeof(unsigned long long));
  const int n = 1 << 24;
  hipLaunchKernelGGL(rcp_k, dim3(n / 256), dim3(256), 0, 0, n, w);
  unsigned long long h[3];
  hipMemcpy(h, w, sizeof(h), hipMemcpyDeviceToHost);
  printf("max ulp error vs 1.0/d: v_rcp_f64 %llu, +1 Newton %llu, +2 Newton %llu\n", h[0], h[1], h[2]);
  return 0;
}
