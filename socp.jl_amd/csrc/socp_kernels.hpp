// socp_kernels.hpp — internal launch interface between socp_api.hip and the
// kernel instantiations (socp_small_inst.hip).
#pragma once
#include <hip/hip_runtime.h>
#include "socp_small.hpp"

namespace socp {

struct SmallVariant {
  int NQ, NP, MQ;
  const void* kernel;  // socp_small_kernel<NQ,NP,MQ>
  const char* name;
};

// table of compiled register-resident variants, ordered by (NQ, NP, MQ)
const SmallVariant* small_variants(int* count);

}  // namespace socp
