// socp_api.hip — C ABI of libsocp (include/socp.h): contexts, device buffers,
// variant dispatch for the register-resident solver kernel, the device-side
// problem generator.  Host pointers are staged through context-owned device
// buffers; device pointers (SOCP_F_DEVICE_PTRS) are used in place.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/socp.h"
#include "socp_kernels.hpp"
#include "socp_sqr.hpp"

using namespace socp;

static thread_local std::string g_err;
// the persistent kernels pull problem indices from an int32 counter and the
// per-problem launches use one workgroup per problem (grid.x)
static constexpr int64_t kMaxBatch = 0x7fffffff;

static int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
#define HIPCHK(x)                                                                   \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess)                                                           \
      return fail(SOCP_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_));      \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes < 256 ? 256 : bytes;
    if (hipMalloc(&p, want) != hipSuccess) return SOCP_E_NOMEM;
    cap = want;
    return 0;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

struct socp_ctx {
  int device = 0;
  hipStream_t own = nullptr;     // created by socp_ctx_create
  hipStream_t stream = nullptr;  // where work goes: `own`, or the caller's (socp_ctx_set_stream)
  // timing pairs around the solver launches, a ring of NTIME so that a run of
  // launches can be timed without a host synchronisation between them
  // (socp_last_kernel_ms, socp_kernel_times)
  static constexpr int NTIME = 64;
  hipEvent_t tev0[NTIME] = {}, tev1[NTIME] = {};
  int64_t tlaunches = 0;
  hipEvent_t evh = nullptr;                 // stream hand-off (ctx_switch_stream), never a timing event
  int num_cu = 0;
  float last_ms = 0.f;
  const char* last_name = "";
  enum { B_C, B_A, B_B, B_G, B_H, B_SING, B_X, B_Y, B_Z, B_S, B_IT, B_ST, B_RES, B_DX, B_DY,
         B_DZ, B_DS, B_CX, B_CY, B_CZ, B_CS, B_CNT, B_LWS, B_ERR, NB };
  DevBuf buf[NB];
};

extern "C" const char* socp_last_error(void) { return g_err.c_str(); }
#ifdef SOCP_DIAG
extern "C" const char* socp_version(void) { return "socp-mi355x 0.1 (gfx950, diagnostic build: phase stamps, KKT dumps)"; }
#else
extern "C" const char* socp_version(void) { return "socp-mi355x 0.1 (gfx950)"; }
#endif

extern "C" void socp_params_default(socp_params* p) {
  p->maxit = 40;
  p->sigma_exp = 3;
  p->tol = 1e-5;
  p->step = 0.99;
  p->init_eps = 1e-10;
  p->flags = 0;
  p->reserved = 0;
}

static void ctx_free(socp_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  // NULL is the null stream (socp_ctx_set_stream(NULL)): synchronise it too,
  // so no kernel still reads the buffers released below
  (void)hipStreamSynchronize(c->stream);
  if (c->own && c->own != c->stream) (void)hipStreamSynchronize(c->own);
  for (auto& b : c->buf) b.release();
  for (int i = 0; i < socp_ctx::NTIME; ++i) {
    if (c->tev0[i]) (void)hipEventDestroy(c->tev0[i]);
    if (c->tev1[i]) (void)hipEventDestroy(c->tev1[i]);
  }
  if (c->evh) (void)hipEventDestroy(c->evh);
  if (c->own) (void)hipStreamDestroy(c->own);
  delete c;
}

extern "C" int socp_ctx_create(int device, socp_ctx** out) {
  if (!out) return fail(SOCP_E_INVALID, "out is NULL");
  *out = nullptr;
  int ndev = 0;
  HIPCHK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(SOCP_E_INVALID, "bad device index");
  HIPCHK(hipSetDevice(device));
  socp_ctx* c = new socp_ctx();
  c->device = device;
  // every partially created resource is released on an error path
  auto bail = [&](hipError_t e, const char* what) {
    ctx_free(c);
    return fail(SOCP_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
  };
  hipDeviceProp_t prop;
  hipError_t e;
  if ((e = hipGetDeviceProperties(&prop, device)) != hipSuccess) return bail(e, "hipGetDeviceProperties");
  c->num_cu = prop.multiProcessorCount;
  if ((e = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking)) != hipSuccess)
    return bail(e, "hipStreamCreateWithFlags");
  c->stream = c->own;
  for (int i = 0; i < socp_ctx::NTIME; ++i) {
    if ((e = hipEventCreate(&c->tev0[i])) != hipSuccess) return bail(e, "hipEventCreate");
    if ((e = hipEventCreate(&c->tev1[i])) != hipSuccess) return bail(e, "hipEventCreate");
  }
  if ((e = hipEventCreateWithFlags(&c->evh, hipEventDisableTiming)) != hipSuccess) return bail(e, "hipEventCreate");
  *out = c;
  return 0;
}

extern "C" int socp_ctx_destroy(socp_ctx* c) {
  ctx_free(c);
  return 0;
}

static int ctx_switch_stream(socp_ctx* c, hipStream_t s) {
  if (s == c->stream) return 0;
  // work already queued on the old stream stays ordered before what follows
  HIPCHK(hipSetDevice(c->device));
  HIPCHK(hipEventRecord(c->evh, c->stream));
  HIPCHK(hipStreamWaitEvent(s, c->evh, 0));
  c->stream = s;
  return 0;
}

// `stream` is taken literally: NULL is HIP's null (default) stream, which is
// torch's default current stream.
extern "C" int socp_ctx_set_stream(socp_ctx* c, void* stream) {
  if (!c) return fail(SOCP_E_INVALID, "ctx is NULL");
  return ctx_switch_stream(c, (hipStream_t)stream);
}

extern "C" int socp_ctx_reset_stream(socp_ctx* c) {
  if (!c) return fail(SOCP_E_INVALID, "ctx is NULL");
  return ctx_switch_stream(c, c->own);
}

extern "C" int socp_ctx_sync(socp_ctx* c) {
  if (!c) return fail(SOCP_E_INVALID, "ctx is NULL");
  HIPCHK(hipStreamSynchronize(c->stream));
  return 0;
}

extern "C" void* socp_ctx_stream(socp_ctx* c) { return c ? (void*)c->stream : nullptr; }

// the timing pair of the next launch (recorded by timing_begin / timing_end)
static hipError_t timing_begin(socp_ctx* c) {
  return hipEventRecord(c->tev0[c->tlaunches % socp_ctx::NTIME], c->stream);
}
static hipError_t timing_end(socp_ctx* c) {
  const hipError_t e = hipEventRecord(c->tev1[c->tlaunches % socp_ctx::NTIME], c->stream);
  if (e == hipSuccess) ++c->tlaunches;
  return e;
}

extern "C" int socp_last_kernel_ms(socp_ctx* c, float* ms) {
  if (!c || !ms) return fail(SOCP_E_INVALID, "NULL argument");
  if (c->tlaunches == 0) return fail(SOCP_E_INVALID, "no timed launch on this context");
  const int i = (int)((c->tlaunches - 1) % socp_ctx::NTIME);
  HIPCHK(hipEventSynchronize(c->tev1[i]));
  HIPCHK(hipEventElapsedTime(&c->last_ms, c->tev0[i], c->tev1[i]));
  *ms = c->last_ms;
  return 0;
}

extern "C" int socp_kernel_times(socp_ctx* c, float* ms, int n) {
  if (!c || !ms || n < 0) return fail(SOCP_E_INVALID, "NULL argument or n < 0");
  int64_t cnt = c->tlaunches < n ? c->tlaunches : n;
  if (cnt > socp_ctx::NTIME) cnt = socp_ctx::NTIME;
  if (cnt == 0) return 0;
  for (int64_t j = 0; j < cnt; ++j) {
    const int i = (int)((c->tlaunches - cnt + j) % socp_ctx::NTIME);
    // each pair is waited on: the pairs may lie on different streams when the
    // context's stream was switched inside the window (socp_ctx_set_stream)
    HIPCHK(hipEventSynchronize(c->tev1[i]));
    HIPCHK(hipEventElapsedTime(&ms[j], c->tev0[i], c->tev1[i]));
  }
  c->last_ms = ms[cnt - 1];
  return (int)cnt;
}
extern "C" const char* socp_last_kernel_name(socp_ctx* c) { return c ? c->last_name : ""; }

// ---------------------------------------------------------------- checks
static int check_problem(const socp_dims* d, const int32_t* kind, const int32_t* offs,
                         const int32_t* dim, ConeTable* tab, int* degree) {
  if (!d) return fail(SOCP_E_INVALID, "dims is NULL");
  if (d->batch < 0 || d->n <= 0 || d->m < 0 || d->k <= 0 || d->ncones <= 0)
    return fail(SOCP_E_INVALID, "bad dims (need batch>=0, n>0, m>=0, k>0, ncones>0)");
  if (d->batch > kMaxBatch)
    return fail(SOCP_E_INVALID, "batch above 2^31-1 (problem indices are int32 on the device)");
  if (d->ncones > MAXC) return fail(SOCP_E_UNSUPPORTED, "too many cones");
  if (!kind || !offs || !dim) return fail(SOCP_E_INVALID, "cone arrays are NULL");
  int next = 0, deg = 0;
  bool seen_soc = false;
  tab->nc = d->ncones;
  for (int c = 0; c < d->ncones; ++c) {
    if (kind[c] != SOCP_CONE_POC && kind[c] != SOCP_CONE_SOC)
      return fail(SOCP_E_INVALID, "cone kind must be POC(0) or SOC(1)");
    if (offs[c] != next || dim[c] <= 0)
      return fail(SOCP_E_INVALID, "cones must be contiguous from 0 with dim>0 (scalings.jl:102)");
    if (kind[c] == SOCP_CONE_POC && seen_soc)
      return fail(SOCP_E_INVALID, "cones must list POC before SOC (scalings.jl:102)");
    if (kind[c] == SOCP_CONE_SOC) seen_soc = true;
    tab->kind[c] = kind[c];
    tab->offs[c] = offs[c];
    tab->dim[c] = dim[c];
    next += dim[c];
    deg += (kind[c] == SOCP_CONE_POC) ? dim[c] : 1;
  }
  if (next != d->k) return fail(SOCP_E_INVALID, "cone dims must sum to k");
  *degree = deg;
  return 0;
}

static const SmallVariant* pick_variant(int n, int m, int k) {
  int cnt = 0;
  const SmallVariant* v = small_variants(&cnt);
  const SmallVariant* best = nullptr;
  long best_cost = 0;
  for (int i = 0; i < cnt; ++i) {
    if (16 * v[i].NQ < n || 4 * v[i].NP < k || 16 * v[i].MQ < (m > 0 ? m : 1)) continue;
    if (k > KMAX) continue;
    long cost = (long)v[i].NQ * v[i].NQ * v[i].NP * 64 + (long)v[i].MQ * 16;
    if (!best || cost < best_cost) {
      best = &v[i];
      best_cost = cost;
    }
  }
  return best;
}

// The blocked kernel (socp_large.hip): n, m <= 2048.  The problem's vectors live in the 160 KiB LDS of a CU when
// they fit; otherwise (e.g. k = 1000 at n = 512) in the workgroup's slot of the
// HBM workspace (*gv: the GV kernels), with only the problem index in LDS.
static bool large_fits(int n, int m, int k, int nc, size_t* lds_bytes, bool* gv = nullptr, bool xi = false) {
  // Every LDS / vector offset of the kernel (LargeLayout::o_*, total, LV(int))
  // is a 32-bit int and X = W^-1 G (KP x NPAD) is addressed from int row
  // offsets: bound k before the layout is computed in int, so that neither
  // wraps (the layout's size is computed here in int64).
  if (n < 0 || m < 0 || k < 0 || k > LARGE_KMAX) return false;
  {
    const int64_t KP = ((int64_t)k + 15) / 16 * 16, NP = ((int64_t)n + 63) / 64 * 64,
                  MP = ((int64_t)(m > 0 ? m : 1) + 63) / 64 * 64, RW = NP > MP ? NP : MP;
    const int64_t lds_total = 16 * KP + 2 * RW + 1024 + 64 + 8 * RW + 16 * RW + 12 * MAXC + 6 * RW + 5 * RW + 64 + 512;
    if (lds_total > INT32_MAX / 2 || KP * RW > INT32_MAX) return false;
  }
  const LargeLayout L = large_layout(n, m, k);
  // n, m: up to 64 LARGE_NB_MAX_CHOL with Cholesky factors of H and S (wide
  // panels in windows, socp_large.hip panel_chol_wide), in both operation
  // orders (SOCP_F_EXPLICIT_INVERSE forms Li and S^-1 from those factors)
  (void)xi;
  if (L.NPAD > 64 * LARGE_NB_MAX_CHOL || L.MPAD > 64 * LARGE_NB_MAX_CHOL || nc > MAXC) return false;
  size_t lds = (size_t)L.total * sizeof(double);
  const bool g = lds + 64 > 160 * 1024;
  if (g) lds = 64 * sizeof(double);
  if (lds_bytes) *lds_bytes = lds;
  if (gv) *gv = g;
  return true;
}

extern "C" int socp_supported(const socp_dims* d) {
  if (!d) return 0;
  if (pick_variant(d->n, d->m, d->k) != nullptr && d->ncones <= NCS) return 1;
  return large_fits(d->n, d->m, d->k, d->ncones, nullptr) ? 1 : 0;
}

static const char* kUnsupported =
    "dims outside both kernels (register-resident: n, m <= 64, k <= 128, <= 8 cones; "
    "blocked: n, m <= 2048, <= 64 cones, k <= 2^21)";

// ---------------------------------------------------------------- launch
static unsigned long long* g_stamps = nullptr;  // per-phase cycle table (SOCP_DIAG builds)

// 1, 2 or 4 when every cone is 16, 32 or 64 long (each cone is then whole
// 16-lane rows of one 64-element slot), else 0
static int cone_rows_uniform(const ConeTable& t, int nc) {
  const int d = t.dim[0];
  if (d != 16 && d != 32 && d != 64) return 0;
  for (int c = 1; c < nc; ++c)
    if (t.dim[c] != d) return 0;
  return d / 16;
}

static int launch_small(socp_ctx* ctx, SmallArgs& args, const SmallVariant* v) {
  args.al_rows = cone_rows_uniform(args.cones, args.nc);
  size_t lds = small_lds_bytes(v->NQ, v->NP, v->MQ);
  if (lds > 160 * 1024) return fail(SOCP_E_UNSUPPORTED, "LDS footprint too large");
  const bool solver = args.mode == MODE_SOLVE;
  // SOCP_F_EXPLICIT_INVERSE: the sweep variants (m <= 16 shapes; larger m sweep anyway)
  const bool xi = (args.flags & SOCP_F_EXPLICIT_INVERSE) != 0 && v->xi_kernel;
  const void* kern = xi ? (solver ? v->xi_kernel : v->xi_kkt_kernel) : (solver ? v->kernel : v->kkt_kernel);
  if (lds > 64 * 1024)
    HIPCHK(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int per_cu = 0;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 64, lds));
  if (per_cu < 1) per_cu = 1;
  int64_t blocks = (int64_t)ctx->num_cu * per_cu;
  if (blocks > args.B) blocks = args.B;
  if (blocks < 1) blocks = 1;
  HIPCHK(hipMemsetAsync(args.counter, 0, sizeof(int32_t), ctx->stream));
  args.stamps = g_stamps;
  void* kargs[] = {&args};
  HIPCHK(timing_begin(ctx));
  HIPCHK(hipLaunchKernel(kern, dim3((unsigned)blocks), dim3(64), kargs, lds, ctx->stream));
  HIPCHK(timing_end(ctx));
  ctx->last_name = xi ? (solver ? v->xi_name : v->xi_kkt_name) : (solver ? v->name : v->kkt_name);
  return 0;
}

static int launch_large(socp_ctx* ctx, const SmallArgs& a, double* rec = nullptr) {
  size_t lds = 0;
  bool gv = false;
  const bool xi = (a.flags & SOCP_F_EXPLICIT_INVERSE) != 0;
  if (!large_fits(a.n, a.m, a.k, a.nc, &lds, &gv, xi)) return fail(SOCP_E_UNSUPPORTED, kUnsupported);
  const void* kern = large_kernel_ptr(xi, gv);
  HIPCHK(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int per_cu = 0;
  HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 512, lds));
  if (per_cu < 1) return fail(SOCP_E_UNSUPPORTED, "blocked kernel does not fit on a CU");
  int64_t grid = (int64_t)ctx->num_cu * per_cu;
  if (grid > a.B) grid = a.B;
  if (grid < 1) grid = 1;
  const LargeLayout L = large_layout(a.n, a.m, a.k);
  LargeArgs la;
  la.a = a;
  la.a.stamps = g_stamps;
  la.wstride = L.w_total;
  const int rc = ctx->buf[socp_ctx::B_LWS].ensure((size_t)grid * (size_t)L.w_total * sizeof(double));
  if (rc) return fail(rc, "workspace allocation failed");
  la.ws = (double*)ctx->buf[socp_ctx::B_LWS].p;
  la.rec = rec;
  HIPCHK(hipMemsetAsync(a.counter, 0, sizeof(int32_t), ctx->stream));
  void* kargs[] = {&la};
  HIPCHK(timing_begin(ctx));
  HIPCHK(hipLaunchKernel(kern, dim3((unsigned)grid), dim3(512), kargs, lds, ctx->stream));
  HIPCHK(timing_end(ctx));
  ctx->last_name = large_kernel_name(xi, gv);
  return 0;
}

template <class T>
static int stage_in(socp_ctx* ctx, int slot, const T* src, size_t count, bool dev, const T** out) {
  if (!src || count == 0) {
    *out = src;
    return 0;
  }
  if (dev) {
    *out = src;
    return 0;
  }
  int rc = ctx->buf[slot].ensure(count * sizeof(T));
  if (rc) return fail(rc, "device allocation failed");
  HIPCHK(hipMemcpyAsync(ctx->buf[slot].p, src, count * sizeof(T), hipMemcpyHostToDevice, ctx->stream));
  *out = (const T*)ctx->buf[slot].p;
  return 0;
}
template <class T>
static int stage_out(socp_ctx* ctx, int slot, T* user, size_t count, bool dev, bool copy_in,
                     T** out) {
  if (!user || count == 0) {
    *out = user;
    return 0;
  }
  if (dev) {
    *out = user;
    return 0;
  }
  int rc = ctx->buf[slot].ensure(count * sizeof(T));
  if (rc) return fail(rc, "device allocation failed");
  if (copy_in)
    HIPCHK(hipMemcpyAsync(ctx->buf[slot].p, user, count * sizeof(T), hipMemcpyHostToDevice, ctx->stream));
  *out = (T*)ctx->buf[slot].p;
  return 0;
}
template <class T>
static int copy_back(socp_ctx* ctx, T* user, const T* devp, size_t count, bool dev) {
  if (dev || !user || count == 0) return 0;
  HIPCHK(hipMemcpyAsync(user, devp, count * sizeof(T), hipMemcpyDeviceToHost, ctx->stream));
  return 0;
}

#define TRY(x)          \
  do {                  \
    int rc_ = (x);      \
    if (rc_) return rc_; \
  } while (0)

// ------------------------------------------------------- problem dumps
// SOCP_DUMP_DIR=<dir> (env): every batch solve writes the first
// SOCP_DUMP_COUNT (default 1) problems of the batch as text, one file per
// quantity, as the reference's commented-out dumps do (solver.jl:48-67: A, G,
// c, b, h, cones; :75-82: the init right-hand side initv = [-c; b; h]).
// Matrices are written one row per line.  Diagnostic only: it synchronises.
static void dump_mat(const char* dir, int64_t p, const char* name, const double* v, int rows, int cols) {
  char fn[1024];
  snprintf(fn, sizeof(fn), "%s/problem%lld_%s.txt", dir, (long long)p, name);
  FILE* f = fopen(fn, "w");
  if (!f) return;
  for (int i = 0; i < rows; ++i) {
    for (int j = 0; j < cols; ++j) fprintf(f, j ? " %.17g" : "%.17g", v[(size_t)j * rows + i]);
    fputc('\n', f);
  }
  fclose(f);
}
static int dump_problems(socp_ctx* ctx, const SmallArgs& a) {
  const char* dir = getenv("SOCP_DUMP_DIR");
  if (!dir || !*dir) return 0;
  const char* cnt = getenv("SOCP_DUMP_COUNT");
  int64_t np = cnt ? atoll(cnt) : 1;
  if (np > a.B) np = a.B;
  const int n = a.n, m = a.m, k = a.k;
  std::vector<double> buf((size_t)k * n + (size_t)m * n + n + m + k + n + m + k);
  HIPCHK(hipStreamSynchronize(ctx->stream));
  for (int64_t p = 0; p < np; ++p) {
    double* G = buf.data();
    double* A = G + (size_t)k * n;
    double* c = A + (size_t)m * n;
    double* b = c + n;
    double* h = b + m;
    double* iv = h + k;
    HIPCHK(hipMemcpy(G, a.G + p * (int64_t)k * n, sizeof(double) * k * n, hipMemcpyDefault));
    if (m) HIPCHK(hipMemcpy(A, a.A + p * (int64_t)m * n, sizeof(double) * m * n, hipMemcpyDefault));
    HIPCHK(hipMemcpy(c, a.c + p * n, sizeof(double) * n, hipMemcpyDefault));
    if (m) HIPCHK(hipMemcpy(b, a.b + p * m, sizeof(double) * m, hipMemcpyDefault));
    HIPCHK(hipMemcpy(h, a.h + p * k, sizeof(double) * k, hipMemcpyDefault));
    for (int j = 0; j < n; ++j) iv[j] = -c[j];
    for (int i = 0; i < m; ++i) iv[n + i] = b[i];
    for (int i = 0; i < k; ++i) iv[n + m + i] = h[i];
    dump_mat(dir, p, "A", A, m, n);
    dump_mat(dir, p, "G", G, k, n);
    dump_mat(dir, p, "c", c, n, 1);
    dump_mat(dir, p, "b", b, m, 1);
    dump_mat(dir, p, "h", h, k, 1);
    dump_mat(dir, p, "initv", iv, n + m + k, 1);
    char fn[1024];
    snprintf(fn, sizeof(fn), "%s/problem%lld_cones.txt", dir, (long long)p);
    if (FILE* f = fopen(fn, "w")) {
      for (int q = 0; q < a.nc; ++q)
        fprintf(f, "%s(%d,%d)\n", a.cones.kind[q] == POC_K ? "POC" : "SOC", a.cones.offs[q], a.cones.dim[q]);
      fclose(f);
    }
  }
  return 0;
}

extern "C" int socp_batch_solve_ex(socp_ctx* ctx, const socp_dims* dims, const int32_t* cone_kind,
                                   const int32_t* cone_offs, const int32_t* cone_dim,
                                   const double* c, const double* A, const double* b,
                                   const double* G, const double* h, const uint8_t* sing,
                                   const socp_params* params, double* x, double* y, double* z,
                                   double* s, int32_t* iters, int32_t* status, double* res) {
  if (!ctx) return fail(SOCP_E_INVALID, "ctx is NULL");
  SmallArgs a;
  memset(&a, 0, sizeof(a));
  int degree = 0;
  TRY(check_problem(dims, cone_kind, cone_offs, cone_dim, &a.cones, &degree));
  socp_params P;
  if (params)
    P = *params;
  else
    socp_params_default(&P);
  const int64_t B = dims->batch;
  const int n = dims->n, m = dims->m, k = dims->k;
  if (B == 0) return 0;
  if (!c || !G || !h || !x || !z || !s || !iters || !status || (m > 0 && (!A || !b || !y)))
    return fail(SOCP_E_INVALID, "NULL data pointer");
  const bool force_large = (P.flags & SOCP_F_FORCE_LARGE) != 0;
  const SmallVariant* v = (force_large || dims->ncones > NCS) ? nullptr : pick_variant(n, m, k);
  if (!v && !large_fits(n, m, k, dims->ncones, nullptr, nullptr, (P.flags & SOCP_F_EXPLICIT_INVERSE) != 0))
    return fail(SOCP_E_UNSUPPORTED, kUnsupported);
  HIPCHK(hipSetDevice(ctx->device));
  const bool dev = (P.flags & SOCP_F_DEVICE_PTRS) != 0;
  const bool warm = (P.flags & SOCP_F_WARM_START) != 0;
  a.B = B;
  a.n = n;
  a.m = m;
  a.k = k;
  a.nc = dims->ncones;
  a.maxit = P.maxit;
  a.sigma_exp = P.sigma_exp;
  a.tol = P.tol;
  a.step = P.step;
  a.init_eps = P.init_eps;
  a.flags = P.flags;
  a.mode = MODE_SOLVE;
  a.deg = degree;
  typedef socp_ctx X;
  TRY(stage_in(ctx, X::B_C, c, (size_t)B * n, dev, &a.c));
  TRY(stage_in(ctx, X::B_A, A, (size_t)B * m * n, dev, &a.A));
  TRY(stage_in(ctx, X::B_B, b, (size_t)B * m, dev, &a.b));
  TRY(stage_in(ctx, X::B_G, G, (size_t)B * k * n, dev, &a.G));
  TRY(stage_in(ctx, X::B_H, h, (size_t)B * k, dev, &a.h));
  TRY(stage_in(ctx, X::B_SING, sing, (size_t)B, dev, &a.sing));
  TRY(stage_out(ctx, X::B_X, x, (size_t)B * n, dev, warm, &a.x));
  TRY(stage_out(ctx, X::B_Y, y, (size_t)B * m, dev, warm, &a.y));
  TRY(stage_out(ctx, X::B_Z, z, (size_t)B * k, dev, warm, &a.z));
  TRY(stage_out(ctx, X::B_S, s, (size_t)B * k, dev, warm, &a.s));
  TRY(stage_out(ctx, X::B_IT, iters, (size_t)B, dev, false, &a.iters));
  TRY(stage_out(ctx, X::B_ST, status, (size_t)B, dev, false, &a.status));
  TRY(stage_out(ctx, X::B_RES, res, (size_t)B * 3, dev, false, &a.res));
  if (ctx->buf[X::B_CNT].ensure(256)) return fail(SOCP_E_NOMEM, "device allocation failed");
  a.counter = (int32_t*)ctx->buf[X::B_CNT].p;
  TRY(dump_problems(ctx, a));
  TRY(v ? launch_small(ctx, a, v) : launch_large(ctx, a));
  TRY(copy_back(ctx, x, a.x, (size_t)B * n, dev));
  TRY(copy_back(ctx, y, a.y, (size_t)B * m, dev));
  TRY(copy_back(ctx, z, a.z, (size_t)B * k, dev));
  TRY(copy_back(ctx, s, a.s, (size_t)B * k, dev));
  TRY(copy_back(ctx, iters, a.iters, (size_t)B, dev));
  TRY(copy_back(ctx, status, a.status, (size_t)B, dev));
  TRY(copy_back(ctx, res, a.res, (size_t)B * 3, dev));
  if (!dev) HIPCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

extern "C" int socp_batch_solve(socp_ctx* ctx, const socp_dims* dims, const int32_t* cone_kind,
                                const int32_t* cone_offs, const int32_t* cone_dim, const double* c,
                                const double* A, const double* b, const double* G, const double* h,
                                const uint8_t* sing, const socp_params* params, double* x,
                                double* y, double* z, double* s, int32_t* iters, int32_t* status) {
  return socp_batch_solve_ex(ctx, dims, cone_kind, cone_offs, cone_dim, c, A, b, G, h, sing, params,
                             x, y, z, s, iters, status, nullptr);
}

static double* g_kkt_debug = nullptr;  // device buffer for socp_debug_kkt (testing hook)
extern "C" int socp_debug_set_stamps(unsigned long long* dev_buf) {
#ifdef SOCP_DIAG
  g_stamps = dev_buf;
  return 0;
#else
  (void)dev_buf;
  return fail(SOCP_E_UNSUPPORTED, "phase stamps exist only in the diagnostic build (libsocp_diag.so)");
#endif
}

extern "C" int socp_debug_set_kkt_dump(double* dev_buf) {
#ifdef SOCP_DIAG
  g_kkt_debug = dev_buf;
  return 0;
#else
  (void)dev_buf;
  return fail(SOCP_E_UNSUPPORTED, "KKT dumps exist only in the diagnostic build (libsocp_diag.so)");
#endif
}

extern "C" int socp_batch_kkt_solve(socp_ctx* ctx, const socp_dims* dims, const int32_t* cone_kind,
                                    const int32_t* cone_offs, const int32_t* cone_dim,
                                    const double* A, const double* G, const uint8_t* sing,
                                    const double* s, const double* z, const double* dx,
                                    const double* dy, const double* dz, const double* ds,
                                    double* cx, double* cy, double* cz, double* cs,
                                    int32_t* kkt_status, int32_t flags) {
  if (!ctx) return fail(SOCP_E_INVALID, "ctx is NULL");
  SmallArgs a;
  memset(&a, 0, sizeof(a));
  int degree = 0;
  TRY(check_problem(dims, cone_kind, cone_offs, cone_dim, &a.cones, &degree));
  const int64_t B = dims->batch;
  const int n = dims->n, m = dims->m, k = dims->k;
  if (B == 0) return 0;
  if (!G || !s || !z || !dx || !dz || !ds || !cx || !cz || !cs || !kkt_status ||
      (m > 0 && (!A || !dy || !cy)))
    return fail(SOCP_E_INVALID, "NULL data pointer");
  const bool force_large = (flags & SOCP_F_FORCE_LARGE) != 0;
  const SmallVariant* v = (force_large || dims->ncones > NCS) ? nullptr : pick_variant(n, m, k);
  if (!v && !large_fits(n, m, k, dims->ncones, nullptr, nullptr, (flags & SOCP_F_EXPLICIT_INVERSE) != 0))
    return fail(SOCP_E_UNSUPPORTED, kUnsupported);
  HIPCHK(hipSetDevice(ctx->device));
  const bool dev = (flags & SOCP_F_DEVICE_PTRS) != 0;
  a.B = B;
  a.n = n;
  a.m = m;
  a.k = k;
  a.nc = dims->ncones;
  a.mode = MODE_KKT;
  a.flags = flags & SOCP_F_EXPLICIT_INVERSE;
  a.deg = degree;
  a.dbg = g_kkt_debug;
  a.maxit = 1;
  a.sigma_exp = 3;
  typedef socp_ctx X;
  // c, b, h are not used by the KKT entry but the loader reads them: point at zeros
  if (ctx->buf[X::B_C].ensure((size_t)B * (n + m + k) * sizeof(double))) return fail(SOCP_E_NOMEM, "alloc");
  HIPCHK(hipMemsetAsync(ctx->buf[X::B_C].p, 0, (size_t)B * (n + m + k) * sizeof(double), ctx->stream));
  a.c = (const double*)ctx->buf[X::B_C].p;
  a.b = a.c + (size_t)B * n;
  a.h = a.b + (size_t)B * m;
  TRY(stage_in(ctx, X::B_A, A, (size_t)B * m * n, dev, &a.A));
  TRY(stage_in(ctx, X::B_G, G, (size_t)B * k * n, dev, &a.G));
  TRY(stage_in(ctx, X::B_SING, sing, (size_t)B, dev, &a.sing));
  TRY(stage_out(ctx, X::B_S, const_cast<double*>(s), (size_t)B * k, dev, true, &a.s));
  TRY(stage_out(ctx, X::B_Z, const_cast<double*>(z), (size_t)B * k, dev, true, &a.z));
  TRY(stage_in(ctx, X::B_DX, dx, (size_t)B * n, dev, &a.dx));
  TRY(stage_in(ctx, X::B_DY, dy, (size_t)B * m, dev, &a.dy));
  TRY(stage_in(ctx, X::B_DZ, dz, (size_t)B * k, dev, &a.dz));
  TRY(stage_in(ctx, X::B_DS, ds, (size_t)B * k, dev, &a.ds));
  TRY(stage_out(ctx, X::B_CX, cx, (size_t)B * n, dev, false, &a.cx));
  TRY(stage_out(ctx, X::B_CY, cy, (size_t)B * m, dev, false, &a.cy));
  TRY(stage_out(ctx, X::B_CZ, cz, (size_t)B * k, dev, false, &a.cz));
  TRY(stage_out(ctx, X::B_CS, cs, (size_t)B * k, dev, false, &a.cs));
  TRY(stage_out(ctx, X::B_ST, kkt_status, (size_t)B, dev, false, &a.status));
  if (ctx->buf[X::B_CNT].ensure(256)) return fail(SOCP_E_NOMEM, "device allocation failed");
  a.counter = (int32_t*)ctx->buf[X::B_CNT].p;
  TRY(v ? launch_small(ctx, a, v) : launch_large(ctx, a));
  TRY(copy_back(ctx, cx, a.cx, (size_t)B * n, dev));
  TRY(copy_back(ctx, cy, a.cy, (size_t)B * m, dev));
  TRY(copy_back(ctx, cz, a.cz, (size_t)B * k, dev));
  TRY(copy_back(ctx, cs, a.cs, (size_t)B * k, dev));
  TRY(copy_back(ctx, kkt_status, a.status, (size_t)B, dev));
  if (!dev) HIPCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

// -------------------------------------------------------- dense handles
// The reference's solver plugin split (densesolver.jl): the solver object is
// built once per problem (A, G kept), setup_iter (:41-52) factors for the
// current (s, z), and solve_kkt (:54-90) is called twice per iteration against
// that factorisation.  A handle keeps A, G (and sing) resident and one factor
// record per problem; a setup_iter call moves s, z in and a solve_kkt call one
// right-hand side, so per-call H2D traffic is O(n + m + k) per problem.
struct socp_dense {
  socp_ctx* ctx = nullptr;
  SmallArgs a;  // problem part filled at create
  const SmallVariant* v = nullptr;
  int64_t rec_stride = 0;
  bool ready = false;      // setup_iter has run
  int64_t h2d_bytes = 0;   // host-to-device bytes moved by the last call
  enum { D_A, D_G, D_SING, D_ZERO, D_REC, D_S, D_Z, D_DX, D_DY, D_DZ, D_DS, D_CX, D_CY, D_CZ, D_CS,
         D_ST, D_CNT, ND };
  DevBuf buf[ND];
};

static void dense_free(socp_dense* h) {
  if (!h) return;
  (void)hipSetDevice(h->ctx->device);
  (void)hipStreamSynchronize(h->ctx->stream);
  for (auto& b : h->buf) b.release();
  delete h;
}

// copies `count` elements into handle buffer `slot`: from the host (counted in
// h2d_bytes) or, with SOCP_F_DEVICE_PTRS, device to device
template <class T>
static int dense_in(socp_dense* h, int slot, const T* src, size_t count, bool dev, const T** out) {
  if (!src || count == 0) {
    *out = src;
    return 0;
  }
  if (dev) {
    *out = src;
    return 0;
  }
  int rc = h->buf[slot].ensure(count * sizeof(T));
  if (rc) return fail(rc, "device allocation failed");
  HIPCHK(hipMemcpyAsync(h->buf[slot].p, src, count * sizeof(T), hipMemcpyHostToDevice, h->ctx->stream));
  h->h2d_bytes += (int64_t)(count * sizeof(T));
  *out = (const T*)h->buf[slot].p;
  return 0;
}
template <class T>
static int dense_out(socp_dense* h, int slot, T* user, size_t count, bool dev, T** out) {
  if (!user || count == 0 || dev) {
    *out = user;
    return 0;
  }
  int rc = h->buf[slot].ensure(count * sizeof(T));
  if (rc) return fail(rc, "device allocation failed");
  *out = (T*)h->buf[slot].p;
  return 0;
}

extern "C" int socp_dense_create(socp_ctx* ctx, const socp_dims* dims, const int32_t* cone_kind,
                                 const int32_t* cone_offs, const int32_t* cone_dim, const double* A,
                                 const double* G, const uint8_t* sing, int32_t flags, socp_dense** out) {
  if (!out) return fail(SOCP_E_INVALID, "out is NULL");
  *out = nullptr;
  if (!ctx) return fail(SOCP_E_INVALID, "ctx is NULL");
  socp_dense* h = new socp_dense();
  h->ctx = ctx;
  SmallArgs& a = h->a;
  memset(&a, 0, sizeof(a));
  int degree = 0;
  auto bail = [&](int rc) {
    dense_free(h);
    return rc;
  };
  int rc = check_problem(dims, cone_kind, cone_offs, cone_dim, &a.cones, &degree);
  if (rc) return bail(rc);
  const int64_t B = dims->batch;
  const int n = dims->n, m = dims->m, k = dims->k;
  if (B > 0 && (!G || (m > 0 && !A))) return bail(fail(SOCP_E_INVALID, "NULL data pointer"));
  const bool force_large = (flags & SOCP_F_FORCE_LARGE) != 0;
  h->v = (force_large || dims->ncones > NCS) ? nullptr : pick_variant(n, m, k);
  if (!h->v && !large_fits(n, m, k, dims->ncones, nullptr, nullptr, (flags & SOCP_F_EXPLICIT_INVERSE) != 0))
    return bail(fail(SOCP_E_UNSUPPORTED, kUnsupported));
  if (hipSetDevice(ctx->device) != hipSuccess) return bail(fail(SOCP_E_HIP, "hipSetDevice"));
  const bool dev = (flags & SOCP_F_DEVICE_PTRS) != 0;
  a.B = B;
  a.n = n;
  a.m = m;
  a.k = k;
  a.nc = dims->ncones;
  a.deg = degree;
  a.maxit = 1;
  a.sigma_exp = 3;
  a.flags = flags & (SOCP_F_DEVICE_PTRS | SOCP_F_EXPLICIT_INVERSE);
  if (B == 0) {
    *out = h;
    return 0;
  }
  typedef socp_dense D;
  // the handle owns its copies (the caller's device buffers may be reused)
  auto own = [&](int slot, const void* src, size_t bytes) -> int {
    if (!src || bytes == 0) return 0;
    if (h->buf[slot].ensure(bytes)) return fail(SOCP_E_NOMEM, "device allocation failed");
    HIPCHK(hipMemcpyAsync(h->buf[slot].p, src, bytes, dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                          ctx->stream));
    if (!dev) h->h2d_bytes += (int64_t)bytes;
    return 0;
  };
  if ((rc = own(D::D_A, A, (size_t)B * m * n * sizeof(double)))) return bail(rc);
  if ((rc = own(D::D_G, G, (size_t)B * k * n * sizeof(double)))) return bail(rc);
  if ((rc = own(D::D_SING, sing, (size_t)B))) return bail(rc);
  a.A = m > 0 ? (const double*)h->buf[D::D_A].p : nullptr;
  a.G = (const double*)h->buf[D::D_G].p;
  a.sing = sing ? (const uint8_t*)h->buf[D::D_SING].p : nullptr;
  // c, b, h are not used by setup_iter / solve_kkt but the loader reads them
  const size_t zb = (size_t)B * (n + m + k) * sizeof(double);
  if (h->buf[D::D_ZERO].ensure(zb)) return bail(fail(SOCP_E_NOMEM, "device allocation failed"));
  if (hipMemsetAsync(h->buf[D::D_ZERO].p, 0, zb, ctx->stream) != hipSuccess)
    return bail(fail(SOCP_E_HIP, "hipMemsetAsync"));
  a.c = (const double*)h->buf[D::D_ZERO].p;
  a.b = a.c + (size_t)B * n;
  a.h = a.b + (size_t)B * m;
  h->rec_stride = h->v ? small_rec_doubles(h->v->NQ, h->v->NP, h->v->MQ) : large_layout(n, m, k).r_total;
  if (h->buf[D::D_REC].ensure((size_t)B * (size_t)h->rec_stride * sizeof(double)))
    return bail(fail(SOCP_E_NOMEM, "factor record allocation failed"));
  if (h->buf[D::D_CNT].ensure(256)) return bail(fail(SOCP_E_NOMEM, "device allocation failed"));
  a.counter = (int32_t*)h->buf[D::D_CNT].p;
  a.rec = (double*)h->buf[D::D_REC].p;
  a.rec_stride = h->rec_stride;
  // host sources may be pageable temporaries the caller frees on return
  if (!dev && hipStreamSynchronize(ctx->stream) != hipSuccess) return bail(fail(SOCP_E_HIP, "hipStreamSynchronize"));
  *out = h;
  return 0;
}

extern "C" int socp_dense_destroy(socp_dense* h) {
  dense_free(h);
  return 0;
}

static int dense_launch(socp_dense* h, SmallArgs& a) {
  return h->v ? launch_small(h->ctx, a, h->v) : launch_large(h->ctx, a, a.rec);
}

extern "C" int socp_dense_setup_iter(socp_dense* h, const double* s, const double* z, int32_t* status) {
  if (!h) return fail(SOCP_E_INVALID, "handle is NULL");
  h->h2d_bytes = 0;
  SmallArgs a = h->a;
  const int64_t B = a.B;
  if (B == 0) {
    h->ready = true;
    return 0;
  }
  if (!s || !z || !status) return fail(SOCP_E_INVALID, "NULL data pointer");
  socp_ctx* ctx = h->ctx;
  HIPCHK(hipSetDevice(ctx->device));
  const bool dev = (a.flags & SOCP_F_DEVICE_PTRS) != 0;
  typedef socp_dense D;
  const size_t k = (size_t)a.k;
  const double *ds_, *dz_;
  TRY(dense_in(h, D::D_S, s, (size_t)B * k, dev, &ds_));
  TRY(dense_in(h, D::D_Z, z, (size_t)B * k, dev, &dz_));
  a.s = const_cast<double*>(ds_);  // read only in MODE_SETUP
  a.z = const_cast<double*>(dz_);
  TRY(dense_out(h, D::D_ST, status, (size_t)B, dev, &a.status));
  a.mode = MODE_SETUP;
  TRY(dense_launch(h, a));
  TRY(copy_back(ctx, status, a.status, (size_t)B, dev));
  if (!dev) HIPCHK(hipStreamSynchronize(ctx->stream));
  h->ready = true;
  return 0;
}

extern "C" int socp_dense_solve_kkt(socp_dense* h, const double* dx, const double* dy, const double* dz,
                                    const double* ds, double* cx, double* cy, double* cz, double* cs,
                                    int32_t* status) {
  if (!h) return fail(SOCP_E_INVALID, "handle is NULL");
  if (!h->ready) return fail(SOCP_E_INVALID, "solve_kkt before setup_iter");
  h->h2d_bytes = 0;
  SmallArgs a = h->a;
  const int64_t B = a.B;
  if (B == 0) return 0;
  const int n = a.n, m = a.m, k = a.k;
  if (!dx || !dz || !ds || !cx || !cz || !cs || !status || (m > 0 && (!dy || !cy)))
    return fail(SOCP_E_INVALID, "NULL data pointer");
  socp_ctx* ctx = h->ctx;
  HIPCHK(hipSetDevice(ctx->device));
  const bool dev = (a.flags & SOCP_F_DEVICE_PTRS) != 0;
  typedef socp_dense D;
  TRY(dense_in(h, D::D_DX, dx, (size_t)B * n, dev, &a.dx));
  TRY(dense_in(h, D::D_DY, dy, (size_t)B * m, dev, &a.dy));
  TRY(dense_in(h, D::D_DZ, dz, (size_t)B * k, dev, &a.dz));
  TRY(dense_in(h, D::D_DS, ds, (size_t)B * k, dev, &a.ds));
  TRY(dense_out(h, D::D_CX, cx, (size_t)B * n, dev, &a.cx));
  TRY(dense_out(h, D::D_CY, cy, (size_t)B * m, dev, &a.cy));
  TRY(dense_out(h, D::D_CZ, cz, (size_t)B * k, dev, &a.cz));
  TRY(dense_out(h, D::D_CS, cs, (size_t)B * k, dev, &a.cs));
  TRY(dense_out(h, D::D_ST, status, (size_t)B, dev, &a.status));
  a.mode = MODE_SOLVEKKT;
  TRY(dense_launch(h, a));
  TRY(copy_back(ctx, cx, a.cx, (size_t)B * n, dev));
  TRY(copy_back(ctx, cy, a.cy, (size_t)B * m, dev));
  TRY(copy_back(ctx, cz, a.cz, (size_t)B * k, dev));
  TRY(copy_back(ctx, cs, a.cs, (size_t)B * k, dev));
  TRY(copy_back(ctx, status, a.status, (size_t)B, dev));
  if (!dev) HIPCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

extern "C" int socp_dense_h2d_bytes(const socp_dense* h, int64_t* bytes) {
  if (!h || !bytes) return fail(SOCP_E_INVALID, "NULL argument");
  *bytes = h->h2d_bytes;
  return 0;
}

extern "C" int64_t socp_dense_record_bytes(const socp_dense* h) {
  return h ? h->rec_stride * (int64_t)sizeof(double) : 0;
}

// ------------------------------------------------------ rank-update handles
// SparseSolver (spsolver.jl:1-130) with SqrScaling (sqrscalings.jl): the
// handle keeps A, G (and sing) on the device, setup_iter computes W^-2 =
// D + uu' - vv', factors G'DG (+A'A), applies the rank-1 modifications and
// factors S into one record per problem; solve_kkt solves against it
// (socp_sqr.hip).
struct socp_sqr {
  socp_ctx* ctx = nullptr;
  SqrArgs a;
  SqrLayout L;
  size_t lds = 0;
  bool dev = false, ready = false;
  int64_t h2d_bytes = 0;
  int deg = 0;  // deg(cones) (vectors.jl:165-179), for mu = lam'lam / deg in solve_socp
  enum { Q_A, Q_G, Q_SING, Q_REC, Q_S, Q_Z, Q_DX, Q_DY, Q_DZ, Q_DS, Q_CX, Q_CY, Q_CZ, Q_CS, Q_ST, Q_OUT,
         Q_IPM, NQB };
  DevBuf buf[NQB];
};

static void sqr_free(socp_sqr* h) {
  if (!h) return;
  (void)hipSetDevice(h->ctx->device);
  (void)hipStreamSynchronize(h->ctx->stream);
  for (auto& b : h->buf) b.release();
  delete h;
}

static bool sqr_fits(const socp_dims* d, size_t* lds) {
  if (d->n < 0 || d->m < 0 || d->k < 0 || d->n > SQR_LMAX || d->m > SQR_LMAX || d->k > SQR_KMAX) return false;
  const size_t bytes = (size_t)sqr_layout(d->n, d->m, d->k, d->ncones).total * sizeof(double);
  if (lds) *lds = bytes;
  return bytes <= 160 * 1024;
}

extern "C" int socp_sqr_supported(const socp_dims* d) { return d && sqr_fits(d, nullptr) ? 1 : 0; }

template <class T>
static int sqr_in(socp_sqr* h, int slot, const T* src, size_t count, const T** out) {
  if (!src || count == 0 || h->dev) {
    *out = src;
    return 0;
  }
  if (h->buf[slot].ensure(count * sizeof(T))) return fail(SOCP_E_NOMEM, "device allocation failed");
  HIPCHK(hipMemcpyAsync(h->buf[slot].p, src, count * sizeof(T), hipMemcpyHostToDevice, h->ctx->stream));
  h->h2d_bytes += (int64_t)(count * sizeof(T));
  *out = (const T*)h->buf[slot].p;
  return 0;
}
template <class T>
static int sqr_out(socp_sqr* h, int slot, T* user, size_t count, T** out) {
  if (!user || count == 0 || h->dev) {
    *out = user;
    return 0;
  }
  if (h->buf[slot].ensure(count * sizeof(T))) return fail(SOCP_E_NOMEM, "device allocation failed");
  *out = (T*)h->buf[slot].p;
  return 0;
}

extern "C" int socp_sqr_create(socp_ctx* ctx, const socp_dims* dims, const int32_t* cone_kind,
                               const int32_t* cone_offs, const int32_t* cone_dim, const double* A,
                               const double* G, const uint8_t* sing, int32_t flags, socp_sqr** out) {
  if (!out) return fail(SOCP_E_INVALID, "out is NULL");
  *out = nullptr;
  if (!ctx) return fail(SOCP_E_INVALID, "ctx is NULL");
  socp_sqr* h = new socp_sqr();
  h->ctx = ctx;
  SqrArgs& a = h->a;
  memset(&a, 0, sizeof(a));
  auto bail = [&](int rc) {
    sqr_free(h);
    return rc;
  };
  int degree = 0;
  int rc = check_problem(dims, cone_kind, cone_offs, cone_dim, &a.cones, &degree);
  if (rc) return bail(rc);
  h->deg = degree;
  if (!sqr_fits(dims, &h->lds))
    return bail(fail(SOCP_E_UNSUPPORTED, "rank-update plugin: n, m <= 1024, k <= 4096, LDS layout <= 160 KiB (socp_sqr.hip)"));
  const int64_t B = dims->batch;
  const int n = dims->n, m = dims->m, k = dims->k;
  if (B > 0 && (!G || (m > 0 && !A))) return bail(fail(SOCP_E_INVALID, "NULL data pointer"));
  if (hipSetDevice(ctx->device) != hipSuccess) return bail(fail(SOCP_E_HIP, "hipSetDevice"));
  h->dev = (flags & SOCP_F_DEVICE_PTRS) != 0;
  a.B = B;
  a.n = n;
  a.m = m;
  a.k = k;
  a.nc = dims->ncones;
  h->L = sqr_layout(n, m, k, a.nc);
  if (B == 0) {
    *out = h;
    return 0;
  }
  typedef socp_sqr Q;
  auto own = [&](int slot, const void* src, size_t bytes) -> int {
    if (!src || bytes == 0) return 0;
    if (h->buf[slot].ensure(bytes)) return fail(SOCP_E_NOMEM, "device allocation failed");
    HIPCHK(hipMemcpyAsync(h->buf[slot].p, src, bytes, h->dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                          ctx->stream));
    if (!h->dev) h->h2d_bytes += (int64_t)bytes;
    return 0;
  };
  if ((rc = own(Q::Q_A, A, (size_t)B * m * n * sizeof(double)))) return bail(rc);
  if ((rc = own(Q::Q_G, G, (size_t)B * k * n * sizeof(double)))) return bail(rc);
  if ((rc = own(Q::Q_SING, sing, (size_t)B))) return bail(rc);
  a.A = m > 0 ? (const double*)h->buf[Q::Q_A].p : nullptr;
  a.G = (const double*)h->buf[Q::Q_G].p;
  a.sing = sing ? (const uint8_t*)h->buf[Q::Q_SING].p : nullptr;
  if (h->buf[Q::Q_REC].ensure((size_t)B * (size_t)h->L.rec * sizeof(double)))
    return bail(fail(SOCP_E_NOMEM, "factor record allocation failed"));
  a.rec = (double*)h->buf[Q::Q_REC].p;
  // the setup kernels write only the factors' lower triangles
  if (hipMemsetAsync(a.rec, 0, (size_t)B * (size_t)h->L.rec * sizeof(double), ctx->stream) != hipSuccess)
    return bail(fail(SOCP_E_HIP, "hipMemsetAsync"));
  const void* kerns[2] = {sqr_setup_kernel_ptr(n, m), sqr_solve_kernel_ptr(n, m)};
  for (const void* kern : kerns)
    if (h->lds > 64 * 1024 &&
        hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)h->lds) != hipSuccess)
      return bail(fail(SOCP_E_HIP, "hipFuncSetAttribute"));
  // host sources may be pageable temporaries the caller frees on return
  if (!h->dev && hipStreamSynchronize(ctx->stream) != hipSuccess)
    return bail(fail(SOCP_E_HIP, "hipStreamSynchronize"));
  *out = h;
  return 0;
}

extern "C" int socp_sqr_destroy(socp_sqr* h) {
  sqr_free(h);
  return 0;
}

static int sqr_launch(socp_sqr* h, const SqrArgs& a, bool setup, bool timed = true) {
  socp_ctx* ctx = h->ctx;
  const void* kern = setup ? sqr_setup_kernel_ptr(a.n, a.m) : sqr_solve_kernel_ptr(a.n, a.m);
  SqrArgs la = a;
  la.stamps = g_stamps;
  void* kargs[] = {&la};
  if (timed) HIPCHK(timing_begin(ctx));
  const int nt = sqr_block_threads(a.n, a.m);
  size_t lds = h->lds;
  if (!setup && nt == 64) {  // the wave solve kernel's own layout (sqr_solve_layout)
    const SqrLayout Ls = sqr_solve_layout(a.n, a.m, a.k, a.nc);
    if (!Ls.large) lds = (size_t)Ls.total * sizeof(double);
  }
  HIPCHK(hipLaunchKernel(kern, dim3((unsigned)a.B), dim3(nt), kargs, lds, ctx->stream));
  if (timed) HIPCHK(timing_end(ctx));
  ctx->last_name = nt > 64 ? (setup ? "socp_sqr_setup_wg_kernel" : "socp_sqr_solve_wg_kernel")
                           : (setup ? "socp_sqr_setup_kernel" : "socp_sqr_solve_kernel");
  return 0;
}

extern "C" int socp_sqr_setup_iter(socp_sqr* h, const double* s, const double* z, int32_t* status) {
  if (!h) return fail(SOCP_E_INVALID, "handle is NULL");
  h->h2d_bytes = 0;
  SqrArgs a = h->a;
  const int64_t B = a.B;
  if (B == 0) {
    h->ready = true;
    return 0;
  }
  if (!s || !z || !status) return fail(SOCP_E_INVALID, "NULL data pointer");
  socp_ctx* ctx = h->ctx;
  HIPCHK(hipSetDevice(ctx->device));
  typedef socp_sqr Q;
  const size_t k = (size_t)a.k;
  TRY(sqr_in(h, Q::Q_S, s, (size_t)B * k, &a.s));
  TRY(sqr_in(h, Q::Q_Z, z, (size_t)B * k, &a.z));
  TRY(sqr_out(h, Q::Q_ST, status, (size_t)B, &a.status));
  TRY(sqr_launch(h, a, true));
  if (!h->dev) {
    HIPCHK(hipMemcpyAsync(status, a.status, (size_t)B * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(hipStreamSynchronize(ctx->stream));
  }
  h->ready = true;
  return 0;
}

extern "C" int socp_sqr_solve_kkt(socp_sqr* h, const double* dx, const double* dy, const double* dz,
                                  const double* ds, double* cx, double* cy, double* cz, double* cs,
                                  int32_t* status) {
  if (!h) return fail(SOCP_E_INVALID, "handle is NULL");
  if (!h->ready) return fail(SOCP_E_INVALID, "solve_kkt before setup_iter");
  h->h2d_bytes = 0;
  SqrArgs a = h->a;
  const int64_t B = a.B;
  if (B == 0) return 0;
  const int n = a.n, m = a.m, k = a.k;
  if (!dx || !dz || !ds || !cx || !cz || !cs || !status || (m > 0 && (!dy || !cy)))
    return fail(SOCP_E_INVALID, "NULL data pointer");
  socp_ctx* ctx = h->ctx;
  HIPCHK(hipSetDevice(ctx->device));
  typedef socp_sqr Q;
  TRY(sqr_in(h, Q::Q_DX, dx, (size_t)B * n, &a.dx));
  TRY(sqr_in(h, Q::Q_DY, dy, (size_t)B * m, &a.dy));
  TRY(sqr_in(h, Q::Q_DZ, dz, (size_t)B * k, &a.dz));
  TRY(sqr_in(h, Q::Q_DS, ds, (size_t)B * k, &a.ds));
  TRY(sqr_out(h, Q::Q_CX, cx, (size_t)B * n, &a.cx));
  TRY(sqr_out(h, Q::Q_CY, cy, (size_t)B * m, &a.cy));
  TRY(sqr_out(h, Q::Q_CZ, cz, (size_t)B * k, &a.cz));
  TRY(sqr_out(h, Q::Q_CS, cs, (size_t)B * k, &a.cs));
  TRY(sqr_out(h, Q::Q_ST, status, (size_t)B, &a.status));
  TRY(sqr_launch(h, a, false));
  TRY(copy_back(ctx, cx, a.cx, (size_t)B * n, h->dev));
  TRY(copy_back(ctx, cy, a.cy, (size_t)B * m, h->dev));
  TRY(copy_back(ctx, cz, a.cz, (size_t)B * k, h->dev));
  TRY(copy_back(ctx, cs, a.cs, (size_t)B * k, h->dev));
  TRY(copy_back(ctx, status, a.status, (size_t)B, h->dev));
  if (!h->dev) HIPCHK(hipStreamSynchronize(ctx->stream));
  return 0;
}

// solve_socp(prob, SolverState(prob, SparseSolver(prob))) (solver.jl:40-153)
// for the handle's whole batch: the initial point, then up to maxit iterations
// of setup_iter + two solve_kkt with this plugin, every problem masked out of
// the launches once it stops (socp_sqr_ipm.hip).  c, b, h in; x, y, z, s,
// iters, status (and res: ||rd||, ||rp||, z's at the returned iterate, may be
// NULL) out; host or device pointers as the handle's flags say.
#ifndef SQR_FUSE_RESID
#define SQR_FUSE_RESID 1  // 0: the separate residual kernel after every setup launch (A/B builds)
#endif
#ifndef SQR_FUSE_SOLVES
#define SQR_FUSE_SOLVES 1  // the iteration's two solves and step phases in one launch (0: four launches)
#endif
extern "C" int socp_sqr_solve_socp(socp_sqr* h, const double* c, const double* b, const double* hv,
                                   const socp_params* params, double* x, double* y, double* z, double* s,
                                   int32_t* iters, int32_t* status, double* res) {
  if (!h) return fail(SOCP_E_INVALID, "handle is NULL");
  const int64_t B = h->a.B;
  if (B == 0) return 0;
  const int n = h->a.n, m = h->a.m, k = h->a.k;
  if (!c || !hv || !x || !z || !s || !iters || !status || (m > 0 && (!b || !y)))
    return fail(SOCP_E_INVALID, "NULL data pointer");
  socp_params P;
  if (params) P = *params; else socp_params_default(&P);
  if (P.maxit < 0) return fail(SOCP_E_INVALID, "maxit < 0");
  if (sqr_ipm_lds_bytes(n, m, k) > 160 * 1024)
    return fail(SOCP_E_UNSUPPORTED, "socp_sqr_solve_socp: the IPM kernels' vectors (7 k + n + m doubles) exceed 160 KiB");
  socp_ctx* ctx = h->ctx;
  HIPCHK(hipSetDevice(ctx->device));
  h->h2d_bytes = 0;
  // device block: c b h | x y z s | dx dy dz ds | rx ry rz rs | res | status iters active st_setup st_solve
  const size_t nd = (size_t)B * (n + m + k) + 4 * (size_t)B * (n + m + 2 * k) + 3 * (size_t)B;
  const size_t ni = 5 * (size_t)B + 1;
  typedef socp_sqr Q;
  if (h->buf[Q::Q_IPM].ensure(nd * sizeof(double) + ni * sizeof(int32_t)))
    return fail(SOCP_E_NOMEM, "device allocation failed");
  double* d = (double*)h->buf[Q::Q_IPM].p;
  SqrIpmArgs ia;
  memset(&ia, 0, sizeof(ia));
  ia.B = B; ia.n = n; ia.m = m; ia.k = k; ia.nc = h->a.nc; ia.deg = h->deg; ia.sigma_exp = P.sigma_exp;
  ia.cones = h->a.cones;
  ia.A = h->a.A; ia.G = h->a.G;
  double* dc = d;
  double* db = dc + (size_t)B * n;
  double* dh = db + (size_t)B * m;
  double* q = dh + (size_t)B * k;
  auto carve4 = [&](double** o0, double** o1, double** o2, double** o3) {
    *o0 = q; q += (size_t)B * n;
    *o1 = q; q += (size_t)B * m;
    *o2 = q; q += (size_t)B * k;
    *o3 = q; q += (size_t)B * k;
  };
  carve4(&ia.x, &ia.y, &ia.z, &ia.s);
  carve4(&ia.dx, &ia.dy, &ia.dz, &ia.ds);
  carve4(&ia.rx, &ia.ry, &ia.rz, &ia.rs);
  ia.res = q; q += 3 * (size_t)B;
  int32_t* ip = (int32_t*)q;
  ia.status = ip; ia.iters = ip + B; ia.active = ip + 2 * B; ia.st_setup = ip + 3 * B;
  int32_t* st_solve = ip + 4 * B;
  ia.n_active = ip + 5 * B;
  // the active count starts at B, set on the stream (no host round trip)
  HIPCHK(hipMemsetD32Async((hipDeviceptr_t)ia.n_active, (int)B, 1, ctx->stream));
  const bool dev = h->dev;
  if (dev) {
    ia.c = c; ia.b = m ? b : nullptr; ia.h = hv;
  } else {
    HIPCHK(hipMemcpyAsync(dc, c, (size_t)B * n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    if (m) HIPCHK(hipMemcpyAsync(db, b, (size_t)B * m * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(dh, hv, (size_t)B * k * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    h->h2d_bytes += (int64_t)((size_t)B * (n + m + k) * sizeof(double));
    ia.c = dc; ia.b = db; ia.h = dh;
  }
  ia.rec = h->a.rec; ia.rec_stride = h->L.rec; ia.r_l = h->L.r_l; ia.r_wb = h->L.r_wb; ia.r_mu = h->L.r_mu;
  ia.tol = P.tol; ia.step = P.step; ia.init_eps = P.init_eps;
  // the plugin's own launches on the IPM's buffers
  SqrArgs su = h->a;  // setup_iter(s, z)
  su.s = ia.s; su.z = ia.z; su.status = ia.st_setup; su.active = nullptr;
  SqrArgs sv = h->a;  // solve_kkt(dx, dy, dz, ds) -> (rx, ry, rz, rs)
  sv.dx = ia.dx; sv.dy = ia.dy; sv.dz = ia.dz; sv.ds = ia.ds;
  sv.cx = ia.rx; sv.cy = ia.ry; sv.cz = ia.rz; sv.cs = ia.rs; sv.status = st_solve; sv.active = nullptr;
  const size_t lds = sqr_ipm_lds_bytes(n, m, k);
  if (lds > 64 * 1024) {
    // above the default 64 KiB of dynamic LDS every IPM kernel has to opt in,
    // as sqr_create does for the setup / solve kernels
    for (int which = 0; which < 6; ++which)
      HIPCHK(hipFuncSetAttribute(sqr_ipm_kernel_ptr(which), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  }
  const dim3 grid((unsigned)B), blk(64);
  auto ipm = [&](int which, int it) -> int {
    void* args1[] = {&ia};
    void* args2[] = {&ia, &it};
    HIPCHK(hipLaunchKernel(sqr_ipm_kernel_ptr(which), grid, blk, which == 4 ? args2 : args1, lds, ctx->stream));
    return 0;
  };
  HIPCHK(timing_begin(ctx));
  // initial point: the KKT system with W = I (s = z = e), then the shift
  TRY(ipm(0, 0));
  TRY(sqr_launch(h, su, true, false));
  sv.init = 1;
  TRY(sqr_launch(h, sv, false, false));
  sv.init = 0;
  TRY(ipm(1, 0));
  su.active = ia.active;
  sv.active = ia.active;
  // the wavefront setup kernel computes the residuals in its pass over G and
  // takes the resid kernel's exit test and right-hand side (SqrArgs::fuse_resid)
  const bool fuse = !h->L.large && SQR_FUSE_RESID;
  if (fuse) {
    su.fuse_resid = 1;
    su.ix = ia.x; su.iy = ia.y; su.ic = ia.c; su.ib = ia.b; su.ih = ia.h;
    su.odx = ia.dx; su.ody = ia.dy; su.odz = ia.dz; su.ods = ia.ds; su.ores = ia.res;
    su.ostatus = ia.status; su.oactive = ia.active; su.n_active = ia.n_active;
    su.tol = P.tol;
  }
  // the wave shapes run the two solves and both step phases in one launch
  const void* solves = SQR_FUSE_SOLVES ? sqr_ipm_solves_kernel_ptr(n, m) : nullptr;
  size_t solves_lds = 0;
  if (solves) {
    const SqrLayout Ls = sqr_solve_layout(n, m, k, h->a.nc);
    solves_lds = (size_t)Ls.total * sizeof(double);
    if (lds > solves_lds) solves_lds = lds;
    if (solves_lds > 160 * 1024) {
      solves = nullptr;
    } else if (solves_lds > 64 * 1024) {
      HIPCHK(hipFuncSetAttribute(solves, hipFuncAttributeMaxDynamicSharedMemorySize, (int)solves_lds));
    }
  }
  for (int it = 0; it < P.maxit; ++it) {
    TRY(sqr_launch(h, su, true, false));   // compute_scaling + setup_iter (+ fused: the residuals)
    if (!fuse) TRY(ipm(2, it));            // residuals, exit test, affine right-hand side
    if (solves) {
      SqrArgs sl = sv;
      sl.stamps = g_stamps;
      int itv = it;
      void* fargs[] = {&sl, &ia, &itv};
      HIPCHK(hipLaunchKernel(solves, grid, blk, fargs, solves_lds, ctx->stream));
    } else {
      TRY(sqr_launch(h, sv, false, false));  // solve_kkt (affine)
      TRY(ipm(3, it));                       // step, sigma, mu, corrector right-hand side
      TRY(sqr_launch(h, sv, false, false));  // solve_kkt (combined)
      TRY(ipm(4, it));                       // step and update
    }
    // under a stopping rule, look every 4 iterations whether any problem is
    // still iterating: the launches over an all-stopped batch are skipped
    if (P.tol > 0.0 && (it & 3) == 3 && it + 1 < P.maxit) {
      int32_t left = 0;
      HIPCHK(hipMemcpyAsync(&left, ia.n_active, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
      HIPCHK(hipStreamSynchronize(ctx->stream));
      if (left <= 0) break;
    }
  }
  if (res) TRY(ipm(5, 0));
  HIPCHK(timing_end(ctx));
  ctx->last_name = "socp_sqr_solve_socp";
  if (dev) {
    HIPCHK(hipMemcpyAsync(x, ia.x, (size_t)B * n * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
    if (m) HIPCHK(hipMemcpyAsync(y, ia.y, (size_t)B * m * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(z, ia.z, (size_t)B * k * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(s, ia.s, (size_t)B * k * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(iters, ia.iters, (size_t)B * sizeof(int32_t), hipMemcpyDeviceToDevice, ctx->stream));
    HIPCHK(hipMemcpyAsync(status, ia.status, (size_t)B * sizeof(int32_t), hipMemcpyDeviceToDevice, ctx->stream));
    if (res) HIPCHK(hipMemcpyAsync(res, ia.res, 3 * (size_t)B * sizeof(double), hipMemcpyDeviceToDevice, ctx->stream));
  } else {
    TRY(copy_back(ctx, x, (const double*)ia.x, (size_t)B * n, false));
    if (m) TRY(copy_back(ctx, y, (const double*)ia.y, (size_t)B * m, false));
    TRY(copy_back(ctx, z, (const double*)ia.z, (size_t)B * k, false));
    TRY(copy_back(ctx, s, (const double*)ia.s, (size_t)B * k, false));
    TRY(copy_back(ctx, iters, (const int32_t*)ia.iters, (size_t)B, false));
    TRY(copy_back(ctx, status, (const int32_t*)ia.status, (size_t)B, false));
    if (res) TRY(copy_back(ctx, res, (const double*)ia.res, 3 * (size_t)B, false));
    HIPCHK(hipStreamSynchronize(ctx->stream));
  }
  h->ready = true;  // the records hold the last iteration's factorisation
  return 0;
}

// one problem's factor of H after modify_factors! (n x n, column-major, zeros
// above the diagonal) -- the Gfact of spsolver.jl:13 as a dense matrix
extern "C" int socp_sqr_factor(socp_sqr* h, int64_t problem, double* L) {
  if (!h || !L) return fail(SOCP_E_INVALID, "NULL argument");
  if (!h->ready) return fail(SOCP_E_INVALID, "factor before setup_iter");
  if (problem < 0 || problem >= h->a.B) return fail(SOCP_E_INVALID, "problem index out of range");
  HIPCHK(hipSetDevice(h->ctx->device));
  const double* src = h->a.rec + problem * h->L.rec + h->L.r_L;
  HIPCHK(hipMemcpyAsync(L, src, (size_t)h->a.n * h->a.n * sizeof(double), hipMemcpyDefault, h->ctx->stream));
  HIPCHK(hipStreamSynchronize(h->ctx->stream));
  return 0;
}

// lambda (B x k), wb (B x k) and mu (B x ncones) of the last setup_iter: the
// SqrScaling fields l, wbs, mu (sqrscalings.jl:11-16) the driver loop reads
extern "C" int socp_sqr_scaling(socp_sqr* h, double* l, double* wbs, double* mu) {
  if (!h) return fail(SOCP_E_INVALID, "handle is NULL");
  if (!h->ready) return fail(SOCP_E_INVALID, "scaling before setup_iter");
  const int64_t B = h->a.B;
  if (B == 0) return 0;
  HIPCHK(hipSetDevice(h->ctx->device));
  const SqrLayout& L = h->L;
  const int k = h->a.k, nc = h->a.nc;
  const size_t pitch = (size_t)L.rec * sizeof(double);
  if (l)
    HIPCHK(hipMemcpy2DAsync(l, k * sizeof(double), h->a.rec + L.r_l, pitch, k * sizeof(double), B,
                            hipMemcpyDefault, h->ctx->stream));
  if (wbs)
    HIPCHK(hipMemcpy2DAsync(wbs, k * sizeof(double), h->a.rec + L.r_wb, pitch, k * sizeof(double), B,
                            hipMemcpyDefault, h->ctx->stream));
  if (mu)
    HIPCHK(hipMemcpy2DAsync(mu, nc * sizeof(double), h->a.rec + L.r_mu, pitch, nc * sizeof(double), B,
                            hipMemcpyDefault, h->ctx->stream));
  HIPCHK(hipStreamSynchronize(h->ctx->stream));
  return 0;
}

extern "C" int socp_sqr_h2d_bytes(const socp_sqr* h, int64_t* bytes) {
  if (!h || !bytes) return fail(SOCP_E_INVALID, "NULL argument");
  *bytes = h->h2d_bytes;
  return 0;
}

extern "C" int64_t socp_sqr_record_bytes(const socp_sqr* h) {
  return h ? h->L.rec * (int64_t)sizeof(double) : 0;
}

// ------------------------------------------------------------- generator
// u = splitmix64(seed ^ (p<<24 | e)), U = (u>>11)*2^-53,
// p the GLOBAL problem index.  Sequential sums without FMA contraction so the
// CPU restatement (oracle/socp_oracle.c: or_generate) is bit-identical.
namespace {
struct GenArgs {
  int64_t B, first;
  uint64_t seed;
  int32_t n, m, k, nc;
  double *c, *A, *b, *G, *h;
  ConeTable cones;
};

// The generator must round exactly like the oracle (gcc -ffp-contract=off):
// hipcc contracts a*b+c into v_fma_f64 by default, and __dadd_rn/__dmul_rn are
// plain operators, so contraction is switched off for these functions (the
// build uses -ffp-contract=fast-honor-pragmas so the pragma is obeyed).
#pragma clang fp contract(off)
// local operators: the bodies of HIP's __dadd_rn/__dmul_rn lie outside this
// pragma and would still be fused
__device__ __forceinline__ double add_rn(double x, double y) { return x + y; }
__device__ __forceinline__ double sub_rn(double x, double y) { return x - y; }
__device__ __forceinline__ double mul_rn(double x, double y) { return x * y; }
__device__ __forceinline__ double sqrt_rn(double x) { return __builtin_sqrt(x); }

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ double gen_u(uint64_t seed, uint64_t p, uint64_t e) {
  uint64_t u = splitmix64(seed ^ ((p << 24) | e));
  return mul_rn((double)(u >> 11), 0x1.0p-53);
}
__device__ __forceinline__ double gen_sym(uint64_t seed, uint64_t p, uint64_t e) {
  return sub_rn(mul_rn(2.0, gen_u(seed, p, e)), 1.0);
}

__global__ void __launch_bounds__(256) socp_generate_kernel(GenArgs a) {
  extern __shared__ double sh[];
  const int64_t p = blockIdx.x;
  const uint64_t gp = (uint64_t)(a.first + p);
  const int n = a.n, m = a.m, k = a.k;
  double* x0 = sh;
  double* y0 = x0 + n;
  double* s0 = y0 + m;
  double* z0 = s0 + k;
  const uint64_t kn = (uint64_t)k * n, mn = (uint64_t)m * n;
  double* Gp = a.G + p * (int64_t)kn;
  double* Ap = a.A + p * (int64_t)mn;
  for (uint64_t e = threadIdx.x; e < kn; e += blockDim.x) Gp[e] = gen_sym(a.seed, gp, e);
  for (uint64_t e = threadIdx.x; e < mn; e += blockDim.x) Ap[e] = gen_sym(a.seed, gp, kn + e);
  const uint64_t base = kn + mn;
  for (int j = threadIdx.x; j < n; j += blockDim.x) x0[j] = gen_sym(a.seed, gp, base + j);
  for (int i = threadIdx.x; i < m; i += blockDim.x) y0[i] = gen_sym(a.seed, gp, base + n + i);
  const uint64_t base2 = base + n + m;
  for (int i = threadIdx.x; i < k; i += blockDim.x) {
    int c = 0;
    while (!(i >= a.cones.offs[c] && i < a.cones.offs[c] + a.cones.dim[c])) ++c;
    const int o = a.cones.offs[c], d = a.cones.dim[c];
    const uint64_t es = base2 + 2 * (uint64_t)o, ez = es + d;
    if (a.cones.kind[c] == POC_K) {
      s0[i] = add_rn(0.5, gen_u(a.seed, gp, es + (i - o)));
      z0[i] = add_rn(0.5, gen_u(a.seed, gp, ez + (i - o)));
    } else if (i > o) {
      s0[i] = gen_sym(a.seed, gp, es + (i - o - 1));
      z0[i] = gen_sym(a.seed, gp, ez + (i - o - 1));
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < a.nc; c += blockDim.x) {
    if (a.cones.kind[c] != SOC_K) continue;
    const int o = a.cones.offs[c], d = a.cones.dim[c];
    const uint64_t es = base2 + 2 * (uint64_t)o, ez = es + d;
    double qs = 0.0, qz = 0.0;
    for (int i = 1; i < d; ++i) {
      qs = add_rn(qs, mul_rn(s0[o + i], s0[o + i]));
      qz = add_rn(qz, mul_rn(z0[o + i], z0[o + i]));
    }
    s0[o] = add_rn(add_rn(sqrt_rn(qs), 0.5), gen_u(a.seed, gp, es + d - 1));
    z0[o] = add_rn(add_rn(sqrt_rn(qz), 0.5), gen_u(a.seed, gp, ez + d - 1));
  }
  __syncthreads();
  for (int i = threadIdx.x; i < k; i += blockDim.x) {
    double acc = 0.0;
    for (int j = 0; j < n; ++j)
      acc = add_rn(acc, mul_rn(gen_sym(a.seed, gp, (uint64_t)j * k + i), x0[j]));
    a.h[p * k + i] = add_rn(acc, s0[i]);
  }
  for (int i = threadIdx.x; i < m; i += blockDim.x) {
    double acc = 0.0;
    for (int j = 0; j < n; ++j)
      acc = add_rn(acc, mul_rn(gen_sym(a.seed, gp, kn + (uint64_t)j * m + i), x0[j]));
    a.b[p * m + i] = acc;
  }
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    double t = 0.0, u = 0.0;
    for (int i = 0; i < m; ++i)
      t = add_rn(t, mul_rn(gen_sym(a.seed, gp, kn + (uint64_t)j * m + i), y0[i]));
    for (int i = 0; i < k; ++i)
      u = add_rn(u, mul_rn(gen_sym(a.seed, gp, (uint64_t)j * k + i), z0[i]));
    a.c[p * n + j] = -add_rn(t, u);
  }
}
#pragma clang fp contract(on)
}  // namespace

extern "C" int socp_generate(socp_ctx* ctx, const socp_dims* dims, const int32_t* cone_kind,
                             const int32_t* cone_offs, const int32_t* cone_dim, uint64_t seed,
                             int64_t first_problem, double* c, double* A, double* b, double* G,
                             double* h) {
  if (!ctx) return fail(SOCP_E_INVALID, "ctx is NULL");
  GenArgs a;
  memset(&a, 0, sizeof(a));
  int degree = 0;
  TRY(check_problem(dims, cone_kind, cone_offs, cone_dim, &a.cones, &degree));
  if (dims->batch == 0) return 0;
  if (first_problem < 0) return fail(SOCP_E_INVALID, "negative first_problem");
  if (!c || !G || !h || (dims->m > 0 && (!A || !b))) return fail(SOCP_E_INVALID, "NULL data pointer");
  if ((uint64_t)dims->k * dims->n + (uint64_t)dims->m * dims->n + dims->n + dims->m + 2 * dims->k >= (1ull << 24))
    return fail(SOCP_E_UNSUPPORTED, "problem too large for the 24-bit element counter");
  HIPCHK(hipSetDevice(ctx->device));
  a.B = dims->batch;
  a.first = first_problem;
  a.seed = seed;
  a.n = dims->n;
  a.m = dims->m;
  a.k = dims->k;
  a.nc = dims->ncones;
  a.c = c;
  a.A = A;
  a.b = b;
  a.G = G;
  a.h = h;
  size_t sh = sizeof(double) * (size_t)(a.n + a.m + 2 * a.k);
  if (sh > 64 * 1024) return fail(SOCP_E_UNSUPPORTED, "generator LDS too large");
  void* kargs[] = {&a};
  HIPCHK(hipLaunchKernel((const void*)&socp_generate_kernel, dim3((unsigned)a.B), dim3(256), kargs,
                         sh, ctx->stream));
  return 0;
}

// --------------------------------------------------------------- ingest
// socp_pack_csc: one workgroup per problem; the problem's dense block is
// zeroed by the workgroup, then every thread scatters a strided share of the
// nonzeros (column by column: the column of nonzero e is found by a binary
// search of colptr, so the scatter is one pass over nz).  A first pass checks
// that every column's row indices are strictly increasing; a problem where one
// is not (duplicates, or unsorted indices as a hand-built CSC may have) is
// packed a thread per column instead, each column's entries summed in input
// order, so repeated (i, j) entries add up as sparse() does and the result is
// deterministic bit for bit.
namespace {
__device__ __forceinline__ int csc_col(const int64_t* cp, int cols, int64_t base, int64_t e) {
  int lo = 0, hi = cols;  // invariant: cp[lo] - base <= e < cp[hi] - base
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (cp[mid] - base <= e) lo = mid; else hi = mid;
  }
  return lo;
}
__global__ void __launch_bounds__(256) socp_pack_csc_kernel(int32_t rows, int32_t cols, const int64_t* nz_offs,
                                                           const int64_t* colptr, const int64_t* rowval,
                                                           const double* nzval, int64_t base, double* dense,
                                                           int32_t* err) {
  __shared__ int unsorted;
  const int64_t p = blockIdx.x;
  const int64_t rc = (int64_t)rows * cols;
  double* D = dense + p * rc;
  if (threadIdx.x == 0) unsorted = 0;
  for (int64_t e = threadIdx.x; e < rc; e += blockDim.x) D[e] = 0.0;
  const int64_t* cp = colptr + p * (int64_t)(cols + 1);
  const int64_t n0 = nz_offs[p], nnz = nz_offs[p + 1] - n0;
  __syncthreads();
  if (cp[0] - base != 0 || cp[cols] - base != nnz) {
    if (threadIdx.x == 0) atomicOr(err, 1);
    return;
  }
  for (int64_t e = threadIdx.x; e + 1 < nnz; e += blockDim.x) {
    const int j = csc_col(cp, cols, base, e);
    if (e + 1 < cp[j + 1] - base && rowval[n0 + e + 1] <= rowval[n0 + e]) unsorted = 1;
  }
  __syncthreads();
  if (unsorted == 0) {  // canonical CSC (SparseMatrixCSC): one store per nonzero
    for (int64_t e = threadIdx.x; e < nnz; e += blockDim.x) {
      const int j = csc_col(cp, cols, base, e);
      const int64_t i = rowval[n0 + e] - base;
      if (i < 0 || i >= rows) {
        atomicOr(err, 2);
        continue;
      }
      D[(int64_t)j * rows + i] = nzval[n0 + e];
    }
    return;
  }
  // unsorted or duplicate row indices: a thread per column sums its entries in
  // input order (sparse()'s combine), so the result is deterministic bit for bit
  for (int j = threadIdx.x; j < cols; j += blockDim.x) {
    for (int64_t e = cp[j] - base; e < cp[j + 1] - base; ++e) {
      const int64_t i = rowval[n0 + e] - base;
      if (i < 0 || i >= rows) {
        atomicOr(err, 2);
        continue;
      }
      D[(int64_t)j * rows + i] += nzval[n0 + e];
    }
  }
}
}  // namespace

extern "C" int socp_pack_csc(socp_ctx* ctx, int64_t batch, int32_t rows, int32_t cols, const int64_t* nz_offs,
                             const int64_t* colptr, const int64_t* rowval, const double* nzval,
                             int32_t index_base, double* dense) {
  if (!ctx) return fail(SOCP_E_INVALID, "ctx is NULL");
  if (batch < 0 || rows < 0 || cols < 0 || (index_base != 0 && index_base != 1))
    return fail(SOCP_E_INVALID, "bad batch/rows/cols/index_base");
  if (batch > kMaxBatch) return fail(SOCP_E_INVALID, "batch above 2^31-1 (one workgroup per problem)");
  if (batch == 0 || (int64_t)rows * cols == 0) return 0;
  if (!nz_offs || !colptr || !dense) return fail(SOCP_E_INVALID, "NULL pointer");
  HIPCHK(hipSetDevice(ctx->device));
  if (ctx->buf[socp_ctx::B_ERR].ensure(256)) return fail(SOCP_E_NOMEM, "device allocation failed");
  int32_t* err = (int32_t*)ctx->buf[socp_ctx::B_ERR].p;
  HIPCHK(hipMemsetAsync(err, 0, sizeof(int32_t), ctx->stream));
  hipLaunchKernelGGL(socp_pack_csc_kernel, dim3((unsigned)batch), dim3(256), 0, ctx->stream, rows, cols, nz_offs,
                     colptr, rowval, nzval, (int64_t)index_base, dense, err);
  HIPCHK(hipGetLastError());
  int32_t herr = 0;
  HIPCHK(hipMemcpyAsync(&herr, err, sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
  HIPCHK(hipStreamSynchronize(ctx->stream));
  if (herr & 1) return fail(SOCP_E_INVALID, "colptr does not span the problem's nonzeros");
  if (herr & 2) return fail(SOCP_E_INVALID, "row index out of range");
  return 0;
}

// ------------------------------------------------------- pipelined ingest
// socp_ingest: host batches -> pinned staging -> device -> solve -> host, with
// two slots so batch i+1's host-to-device copy (and CSC packing) runs on a copy
// stream while batch i solves on the context's stream, and batch i's results
// drain on a third stream.  Per slot: one pinned input block, one pinned output
// block, device buffers, and three events (inputs on the device, solved,
// outputs on the host).
namespace {
constexpr size_t kAl = 256;
inline size_t al_up(size_t v) { return (v + kAl - 1) / kAl * kAl; }

struct IngestSlot {
  void* pin_in = nullptr;
  void* pin_out = nullptr;
  void* pin_csc = nullptr;  // CSC staging, grown on its own so pin_in never moves
  size_t pin_in_cap = 0, pin_out_cap = 0, pin_csc_cap = 0;
  DevBuf dev_in, dev_out, dev_csc;
  hipEvent_t ready = nullptr, solved = nullptr, done = nullptr;
  int64_t ticket = -1;  // outstanding ticket, -1 when free
  int64_t batch = 0;
  bool csc = false;
};

// parallel host copy into pinned staging (a single thread reaches ~10 GB/s,
// well below PCIe; larger copies are split over up to 8 threads)
void par_copy(void* dst, const void* src, size_t bytes) {
  if (!src || !bytes || dst == src) return;
  const size_t chunk = 64ull << 20;
  const unsigned nt = (unsigned)std::min<size_t>(8, (bytes + chunk - 1) / chunk);
  if (nt <= 1) {
    memcpy(dst, src, bytes);
    return;
  }
  std::vector<std::thread> th;
  const size_t per = (bytes + nt - 1) / nt;
  for (unsigned t = 0; t < nt; ++t) {
    const size_t o = (size_t)t * per;
    if (o >= bytes) break;
    const size_t len = std::min(per, bytes - o);
    th.emplace_back([=] { memcpy((char*)dst + o, (const char*)src + o, len); });
  }
  for (auto& t : th) t.join();
}
}  // namespace

struct socp_ingest {
  socp_ctx* ctx = nullptr;
  socp_dims dims;  // dims.batch = the largest batch a submit may carry
  ConeTable cones;
  int degree = 0;
  int32_t flags = 0;
  const SmallVariant* v = nullptr;
  hipStream_t h2d = nullptr, d2h = nullptr;
  IngestSlot slot[2];
  int64_t next = 0;
  DevBuf counter, err;
};

// the byte layout of one slot's blocks for `B` problems
struct InLayout {
  size_t c, A, b, G, h, sing, total;
};
static InLayout in_layout(const socp_dims& d, int64_t B) {
  InLayout L;
  size_t o = 0;
  L.c = o;    o += al_up(sizeof(double) * B * d.n);
  L.A = o;    o += al_up(sizeof(double) * B * d.m * d.n);
  L.b = o;    o += al_up(sizeof(double) * B * d.m);
  L.G = o;    o += al_up(sizeof(double) * B * d.k * d.n);
  L.h = o;    o += al_up(sizeof(double) * B * d.k);
  L.sing = o; o += al_up((size_t)B);
  L.total = o;
  return L;
}
struct OutLayout {
  size_t x, y, z, s, it, st, res, err, total;
};
static OutLayout out_layout(const socp_dims& d, int64_t B) {
  OutLayout L;
  size_t o = 0;
  L.x = o;   o += al_up(sizeof(double) * B * d.n);
  L.y = o;   o += al_up(sizeof(double) * B * d.m);
  L.z = o;   o += al_up(sizeof(double) * B * d.k);
  L.s = o;   o += al_up(sizeof(double) * B * d.k);
  L.it = o;  o += al_up(sizeof(int32_t) * B);
  L.st = o;  o += al_up(sizeof(int32_t) * B);
  L.res = o; o += al_up(sizeof(double) * 3 * B);
  L.err = o; o += kAl;
  L.total = o;
  return L;
}

static void ingest_free(socp_ingest* g) {
  if (!g) return;
  (void)hipSetDevice(g->ctx->device);
  if (g->h2d) (void)hipStreamSynchronize(g->h2d);
  (void)hipStreamSynchronize(g->ctx->stream);
  if (g->d2h) (void)hipStreamSynchronize(g->d2h);
  for (auto& sl : g->slot) {
    if (sl.pin_in) (void)hipHostFree(sl.pin_in);
    if (sl.pin_out) (void)hipHostFree(sl.pin_out);
    if (sl.pin_csc) (void)hipHostFree(sl.pin_csc);
    sl.dev_in.release();
    sl.dev_out.release();
    sl.dev_csc.release();
    if (sl.ready) (void)hipEventDestroy(sl.ready);
    if (sl.solved) (void)hipEventDestroy(sl.solved);
    if (sl.done) (void)hipEventDestroy(sl.done);
  }
  g->counter.release();
  g->err.release();
  if (g->h2d) (void)hipStreamDestroy(g->h2d);
  if (g->d2h) (void)hipStreamDestroy(g->d2h);
  delete g;
}

extern "C" int socp_ingest_create(socp_ctx* ctx, const socp_dims* dims, const int32_t* cone_kind,
                                  const int32_t* cone_offs, const int32_t* cone_dim, int32_t flags,
                                  socp_ingest** out) {
  if (!out) return fail(SOCP_E_INVALID, "out is NULL");
  *out = nullptr;
  if (!ctx) return fail(SOCP_E_INVALID, "ctx is NULL");
  socp_ingest* g = new socp_ingest();
  g->ctx = ctx;
  auto bail = [&](int rc) {
    ingest_free(g);
    return rc;
  };
  int rc = check_problem(dims, cone_kind, cone_offs, cone_dim, &g->cones, &g->degree);
  if (rc) return bail(rc);
  g->dims = *dims;
  g->flags = flags & SOCP_F_FORCE_LARGE;
  const int n = dims->n, m = dims->m, k = dims->k;
  g->v = ((flags & SOCP_F_FORCE_LARGE) || dims->ncones > NCS) ? nullptr : pick_variant(n, m, k);
  if (!g->v && !large_fits(n, m, k, dims->ncones, nullptr)) return bail(fail(SOCP_E_UNSUPPORTED, kUnsupported));
  hipError_t e;
  if ((e = hipSetDevice(ctx->device)) != hipSuccess) return bail(fail(SOCP_E_HIP, "hipSetDevice"));
  if ((e = hipStreamCreateWithFlags(&g->h2d, hipStreamNonBlocking)) != hipSuccess ||
      (e = hipStreamCreateWithFlags(&g->d2h, hipStreamNonBlocking)) != hipSuccess)
    return bail(fail(SOCP_E_HIP, std::string("hipStreamCreateWithFlags: ") + hipGetErrorString(e)));
  const int64_t B = dims->batch;
  const InLayout Li = in_layout(*dims, B);
  const OutLayout Lo = out_layout(*dims, B);
  for (auto& sl : g->slot) {
    if (hipEventCreateWithFlags(&sl.ready, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&sl.solved, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) != hipSuccess)
      return bail(fail(SOCP_E_HIP, "hipEventCreate"));
    if (hipHostMalloc(&sl.pin_in, Li.total, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&sl.pin_out, Lo.total, hipHostMallocDefault) != hipSuccess)
      return bail(fail(SOCP_E_NOMEM, "pinned host allocation failed"));
    sl.pin_in_cap = Li.total;
    sl.pin_out_cap = Lo.total;
    if (sl.dev_in.ensure(Li.total) || sl.dev_out.ensure(Lo.total))
      return bail(fail(SOCP_E_NOMEM, "device allocation failed"));
  }
  if (g->counter.ensure(256) || g->err.ensure(256)) return bail(fail(SOCP_E_NOMEM, "device allocation failed"));
  *out = g;
  return 0;
}

extern "C" int socp_ingest_destroy(socp_ingest* g) {
  ingest_free(g);
  return 0;
}

// pinned input arrays of the slot the next submit will use: a producer that
// writes there directly saves the host copy (submit sees its own pointers)
extern "C" int socp_ingest_next_inputs(socp_ingest* g, double** c, double** A, double** b, double** G,
                                       double** h, uint8_t** sing) {
  if (!g) return fail(SOCP_E_INVALID, "ingest is NULL");
  IngestSlot& sl = g->slot[g->next & 1];
  if (sl.ticket >= 0) return fail(SOCP_E_INVALID, "the next slot is busy: wait for its ticket first");
  const InLayout L = in_layout(g->dims, g->dims.batch);
  char* base = (char*)sl.pin_in;
  if (c) *c = (double*)(base + L.c);
  if (A) *A = (double*)(base + L.A);
  if (b) *b = (double*)(base + L.b);
  if (G) *G = (double*)(base + L.G);
  if (h) *h = (double*)(base + L.h);
  if (sing) *sing = (uint8_t*)(base + L.sing);
  return 0;
}

// the part of submit shared by the dense and CSC forms: the slot's solve on the
// context's stream after `ready`, and the result copies on the d2h stream
static int ingest_solve(socp_ingest* g, IngestSlot& sl, int64_t B, const uint8_t* sing_dev, bool have_sing,
                        const socp_params* params, const double* A_dev, const double* G_dev) {
  socp_ctx* ctx = g->ctx;
  const socp_dims& d = g->dims;
  const InLayout Li = in_layout(d, d.batch);
  const OutLayout Lo = out_layout(d, d.batch);
  char* din = (char*)sl.dev_in.p;
  char* dout = (char*)sl.dev_out.p;
  socp_params P;
  if (params)
    P = *params;
  else
    socp_params_default(&P);
  SmallArgs a;
  memset(&a, 0, sizeof(a));
  a.cones = g->cones;
  a.B = B;
  a.n = d.n;
  a.m = d.m;
  a.k = d.k;
  a.nc = d.ncones;
  a.maxit = P.maxit;
  a.sigma_exp = P.sigma_exp;
  a.tol = P.tol;
  a.step = P.step;
  a.init_eps = P.init_eps;
  a.flags = P.flags & ~SOCP_F_WARM_START;
  a.mode = MODE_SOLVE;
  a.deg = g->degree;
  a.c = (const double*)(din + Li.c);
  a.A = d.m > 0 ? A_dev : nullptr;
  a.b = (const double*)(din + Li.b);
  a.G = G_dev;
  a.h = (const double*)(din + Li.h);
  a.sing = have_sing ? sing_dev : nullptr;
  a.x = (double*)(dout + Lo.x);
  a.y = (double*)(dout + Lo.y);
  a.z = (double*)(dout + Lo.z);
  a.s = (double*)(dout + Lo.s);
  a.iters = (int32_t*)(dout + Lo.it);
  a.status = (int32_t*)(dout + Lo.st);
  a.res = (double*)(dout + Lo.res);
  a.counter = (int32_t*)g->counter.p;
  HIPCHK(hipStreamWaitEvent(ctx->stream, sl.ready, 0));
  TRY(g->v ? launch_small(ctx, a, g->v) : launch_large(ctx, a));
  HIPCHK(hipEventRecord(sl.solved, ctx->stream));
  HIPCHK(hipStreamWaitEvent(g->d2h, sl.solved, 0));
  // one copy of the whole output block (x y z s iters status res err)
  const size_t used = Lo.total;
  HIPCHK(hipMemcpyAsync(sl.pin_out, dout, used, hipMemcpyDeviceToHost, g->d2h));
  HIPCHK(hipEventRecord(sl.done, g->d2h));
  return 0;
}

static int ingest_begin(socp_ingest* g, int64_t batch, IngestSlot** out) {
  if (!g) return fail(SOCP_E_INVALID, "ingest is NULL");
  if (batch < 0 || batch > g->dims.batch) return fail(SOCP_E_INVALID, "batch outside 0..max_batch of the ingest");
  IngestSlot& sl = g->slot[g->next & 1];
  if (sl.ticket >= 0) return fail(SOCP_E_INVALID, "two tickets outstanding: wait for the older one first");
  HIPCHK(hipSetDevice(g->ctx->device));
  *out = &sl;
  return 0;
}

extern "C" int socp_ingest_submit(socp_ingest* g, int64_t batch, const double* c, const double* A, const double* b,
                                  const double* G, const double* h, const uint8_t* sing, const socp_params* params,
                                  int64_t* ticket) {
  IngestSlot* slp = nullptr;
  TRY(ingest_begin(g, batch, &slp));
  IngestSlot& sl = *slp;
  const socp_dims& d = g->dims;
  const int64_t B = batch;
  if (!ticket) return fail(SOCP_E_INVALID, "ticket is NULL");
  if (B > 0 && (!c || !G || !h || (d.m > 0 && (!A || !b)))) return fail(SOCP_E_INVALID, "NULL data pointer");
  const InLayout L = in_layout(d, d.batch);
  char* pin = (char*)sl.pin_in;
  char* din = (char*)sl.dev_in.p;
  // host -> pinned (skipped for arrays already written into the slot)
  const size_t nb[6] = {sizeof(double) * B * d.n, sizeof(double) * B * d.m * d.n, sizeof(double) * B * d.m,
                        sizeof(double) * B * d.k * d.n, sizeof(double) * B * d.k, (size_t)B};
  const size_t off[6] = {L.c, L.A, L.b, L.G, L.h, L.sing};
  const void* src[6] = {c, A, b, G, h, sing};
  for (int i = 0; i < 6; ++i) par_copy(pin + off[i], src[i], nb[i]);
  // pinned -> device on the copy stream: one transfer per array
  for (int i = 0; i < 6; ++i)
    if (src[i] && nb[i]) HIPCHK(hipMemcpyAsync(din + off[i], pin + off[i], nb[i], hipMemcpyHostToDevice, g->h2d));
  HIPCHK(hipEventRecord(sl.ready, g->h2d));
  if (B > 0)
    TRY(ingest_solve(g, sl, B, (const uint8_t*)(din + L.sing), sing != nullptr, params,
                     (const double*)(din + L.A), (const double*)(din + L.G)));
  sl.ticket = g->next++;
  sl.batch = B;
  sl.csc = false;
  *ticket = sl.ticket;
  return 0;
}

// CSC form: A and G arrive as the SparseMatrixCSC arrays of socp_pack_csc;
// they are copied to the device and packed there on the copy stream
extern "C" int socp_ingest_submit_csc(socp_ingest* g, int64_t batch, const double* c, const double* b,
                                      const double* h, const uint8_t* sing, const int64_t* A_nz_offs,
                                      const int64_t* A_colptr, const int64_t* A_rowval, const double* A_nzval,
                                      const int64_t* G_nz_offs, const int64_t* G_colptr, const int64_t* G_rowval,
                                      const double* G_nzval, int32_t index_base, const socp_params* params,
                                      int64_t* ticket) {
  IngestSlot* slp = nullptr;
  TRY(ingest_begin(g, batch, &slp));
  IngestSlot& sl = *slp;
  const socp_dims& d = g->dims;
  const int64_t B = batch;
  if (!ticket) return fail(SOCP_E_INVALID, "ticket is NULL");
  if (index_base != 0 && index_base != 1) return fail(SOCP_E_INVALID, "index_base must be 0 or 1");
  if (B > 0 && (!c || !h || !G_nz_offs || !G_colptr || (d.m > 0 && (!b || !A_nz_offs || !A_colptr))))
    return fail(SOCP_E_INVALID, "NULL data pointer");
  const InLayout L = in_layout(d, d.batch);
  char* pin = (char*)sl.pin_in;
  char* din = (char*)sl.dev_in.p;
  const size_t nb[4] = {sizeof(double) * B * d.n, sizeof(double) * B * d.m, sizeof(double) * B * d.k, (size_t)B};
  const size_t off[4] = {L.c, L.b, L.h, L.sing};
  const void* src[4] = {c, b, h, sing};
  for (int i = 0; i < 4; ++i) par_copy(pin + off[i], src[i], nb[i]);
  for (int i = 0; i < 4; ++i)
    if (src[i] && nb[i]) HIPCHK(hipMemcpyAsync(din + off[i], pin + off[i], nb[i], hipMemcpyHostToDevice, g->h2d));
  // the CSC arrays: sizes from the host offsets; staged in the slot's own
  // pinned CSC block (grown on demand), so the pinned input block -- and the
  // pointers socp_ingest_next_inputs handed out for it -- never move
  const int64_t nzA = (d.m > 0 && B > 0) ? A_nz_offs[B] - A_nz_offs[0] : 0;
  const int64_t nzG = B > 0 ? G_nz_offs[B] - G_nz_offs[0] : 0;
  if (nzA < 0 || nzG < 0) return fail(SOCP_E_INVALID, "nz_offs must be non-decreasing");
  const size_t cA = (size_t)(d.n + 1), cG = (size_t)(d.n + 1);
  size_t o = 0;
  const size_t oAo = o;  o += al_up(sizeof(int64_t) * (B + 1));
  const size_t oAc = o;  o += al_up(sizeof(int64_t) * B * cA);
  const size_t oAr = o;  o += al_up(sizeof(int64_t) * (nzA + 1));
  const size_t oAv = o;  o += al_up(sizeof(double) * (nzA + 1));
  const size_t oGo = o;  o += al_up(sizeof(int64_t) * (B + 1));
  const size_t oGc = o;  o += al_up(sizeof(int64_t) * B * cG);
  const size_t oGr = o;  o += al_up(sizeof(int64_t) * (nzG + 1));
  const size_t oGv = o;  o += al_up(sizeof(double) * (nzG + 1));
  const size_t csc_bytes = o;
  if (csc_bytes > sl.pin_csc_cap) {
    // the slot is free (ingest_begin); drain the copy stream anyway before
    // the old block goes
    HIPCHK(hipStreamSynchronize(g->h2d));
    if (sl.pin_csc) (void)hipHostFree(sl.pin_csc);
    sl.pin_csc = nullptr;
    sl.pin_csc_cap = 0;
    if (hipHostMalloc(&sl.pin_csc, csc_bytes, hipHostMallocDefault) != hipSuccess)
      return fail(SOCP_E_NOMEM, "pinned host allocation failed");
    sl.pin_csc_cap = csc_bytes;
  }
  // device: the CSC arrays, then the dense A and G they are packed into
  const size_t dA = al_up(sizeof(double) * B * d.m * d.n), dG = al_up(sizeof(double) * B * d.k * d.n);
  if (sl.dev_csc.ensure(csc_bytes + dA + dG)) return fail(SOCP_E_NOMEM, "device allocation failed");
  char* pc = (char*)sl.pin_csc;
  char* dc = (char*)sl.dev_csc.p;
  // offsets are rebased to start at 0 for the pack kernel
  auto put_offs = [&](size_t off_, const int64_t* v) {
    int64_t* t = (int64_t*)(pc + off_);
    for (int64_t p = 0; p <= B; ++p) t[p] = v[p] - v[0];
  };
  if (d.m > 0 && B > 0) {
    put_offs(oAo, A_nz_offs);
    par_copy(pc + oAc, A_colptr, sizeof(int64_t) * B * cA);
    par_copy(pc + oAr, A_rowval + 0, sizeof(int64_t) * nzA);
    par_copy(pc + oAv, A_nzval + 0, sizeof(double) * nzA);
  }
  if (B > 0) {
    put_offs(oGo, G_nz_offs);
    par_copy(pc + oGc, G_colptr, sizeof(int64_t) * B * cG);
    par_copy(pc + oGr, G_rowval, sizeof(int64_t) * nzG);
    par_copy(pc + oGv, G_nzval, sizeof(double) * nzG);
  }
  if (B > 0) HIPCHK(hipMemcpyAsync(dc, pc, csc_bytes, hipMemcpyHostToDevice, g->h2d));
  double* A_dev = (double*)(dc + csc_bytes);
  double* G_dev = (double*)(dc + csc_bytes + dA);
  int32_t* err = (int32_t*)((char*)sl.dev_out.p + out_layout(d, d.batch).err);
  HIPCHK(hipMemsetAsync(err, 0, sizeof(int32_t), g->h2d));
  if (B > 0 && d.m > 0)
    hipLaunchKernelGGL(socp_pack_csc_kernel, dim3((unsigned)B), dim3(256), 0, g->h2d, d.m, d.n,
                       (const int64_t*)(dc + oAo), (const int64_t*)(dc + oAc), (const int64_t*)(dc + oAr),
                       (const double*)(dc + oAv), (int64_t)index_base, A_dev, err);
  if (B > 0)
    hipLaunchKernelGGL(socp_pack_csc_kernel, dim3((unsigned)B), dim3(256), 0, g->h2d, d.k, d.n,
                       (const int64_t*)(dc + oGo), (const int64_t*)(dc + oGc), (const int64_t*)(dc + oGr),
                       (const double*)(dc + oGv), (int64_t)index_base, G_dev, err);
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(sl.ready, g->h2d));
  if (B > 0) TRY(ingest_solve(g, sl, B, (const uint8_t*)(din + L.sing), sing != nullptr, params, A_dev, G_dev));
  sl.ticket = g->next++;
  sl.batch = B;
  sl.csc = true;
  *ticket = sl.ticket;
  return 0;
}

extern "C" int socp_ingest_wait(socp_ingest* g, int64_t ticket, double* x, double* y, double* z, double* s,
                                int32_t* iters, int32_t* status, double* res) {
  if (!g) return fail(SOCP_E_INVALID, "ingest is NULL");
  IngestSlot* slp = nullptr;
  for (auto& sl : g->slot)
    if (sl.ticket == ticket && ticket >= 0) slp = &sl;
  if (!slp) return fail(SOCP_E_INVALID, "unknown or already collected ticket");
  IngestSlot& sl = *slp;
  HIPCHK(hipSetDevice(g->ctx->device));
  sl.ticket = -1;  // the slot is free again whatever happens below
  if (sl.batch == 0) return 0;
  HIPCHK(hipEventSynchronize(sl.done));
  const socp_dims& d = g->dims;
  const int64_t B = sl.batch;
  const OutLayout L = out_layout(d, d.batch);
  const char* po = (const char*)sl.pin_out;
  if (sl.csc) {
    const int32_t herr = *(const int32_t*)(po + L.err);
    if (herr & 1) return fail(SOCP_E_INVALID, "colptr does not span the problem's nonzeros");
    if (herr & 2) return fail(SOCP_E_INVALID, "row index out of range");
  }
  par_copy(x, po + L.x, sizeof(double) * B * d.n);
  if (y) par_copy(y, po + L.y, sizeof(double) * B * d.m);
  par_copy(z, po + L.z, sizeof(double) * B * d.k);
  par_copy(s, po + L.s, sizeof(double) * B * d.k);
  if (iters) memcpy(iters, po + L.it, sizeof(int32_t) * B);
  if (status) memcpy(status, po + L.st, sizeof(int32_t) * B);
  if (res) memcpy(res, po + L.res, sizeof(double) * 3 * B);
  return 0;
}

// ------------------------------------------------------------ multi-GPU gather
// RCCL entry points resolved from librccl.so.1 on first use (a process that
// already loaded it, e.g. through torch, shares that copy: same soname).
namespace {
struct Rccl {
  decltype(&ncclGetUniqueId) get_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclGetErrorString) err_str = nullptr;
  bool ok = false;
};
const Rccl* rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    r.get_id = (decltype(r.get_id))dlsym(h, "ncclGetUniqueId");
    r.init_rank = (decltype(r.init_rank))dlsym(h, "ncclCommInitRank");
    r.destroy = (decltype(r.destroy))dlsym(h, "ncclCommDestroy");
    r.all_gather = (decltype(r.all_gather))dlsym(h, "ncclAllGather");
    r.err_str = (decltype(r.err_str))dlsym(h, "ncclGetErrorString");
    r.ok = r.get_id && r.init_rank && r.destroy && r.all_gather && r.err_str;
  });
  return r.ok ? &r : nullptr;
}

// 32-byte outcome record (include/socp.h socp_outcome): status, iters, and the
// exit-test quantities ||rd||, ||rp||, z's (solver.jl:109-122)
__global__ void socp_outcome_kernel(int64_t B, const int32_t* __restrict__ status, const int32_t* __restrict__ iters,
                                    const double* __restrict__ res, socp_outcome* __restrict__ rec) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < B) {
    socp_outcome o;
    o.status = status[p];
    o.iters = iters[p];
    o.res_dual = res ? res[3 * p] : NAN;
    o.res_primal = res ? res[3 * p + 1] : NAN;
    o.gap = res ? res[3 * p + 2] : NAN;
    rec[p] = o;
  }
}

__global__ void socp_pair_kernel(int64_t B, const int32_t* __restrict__ status, const int32_t* __restrict__ iters,
                                 int32_t* __restrict__ pairs) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < B) {
    pairs[2 * p] = status[p];
    pairs[2 * p + 1] = iters[p];
  }
}
}  // namespace

struct socp_comm {
  socp_ctx* ctx = nullptr;  // must outlive the comm (destroy the comm first)
  int device = 0;
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = 0;
  DevBuf pairs;
};

static_assert(sizeof(ncclUniqueId) == SOCP_COMM_ID_BYTES, "ncclUniqueId size");

#define RCCLCHK(R, x)                                                                       \
  do {                                                                                     \
    ncclResult_t r_ = (x);                                                                 \
    if (r_ != ncclSuccess) return fail(SOCP_E_HIP, std::string(#x) + ": " + (R)->err_str(r_)); \
  } while (0)

extern "C" int socp_comm_unique_id(unsigned char* id) {
  if (!id) return fail(SOCP_E_INVALID, "id is NULL");
  const Rccl* R = rccl();
  if (!R) return fail(SOCP_E_UNSUPPORTED, "librccl.so.1 not found");
  ncclUniqueId u;
  RCCLCHK(R, R->get_id(&u));
  memcpy(id, &u, sizeof(u));
  return 0;
}

extern "C" int socp_comm_init(socp_ctx* ctx, int nranks, int rank, const unsigned char* id, socp_comm** out) {
  if (!ctx || !id || !out) return fail(SOCP_E_INVALID, "NULL argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(SOCP_E_INVALID, "bad nranks/rank");
  const Rccl* R = rccl();
  if (!R) return fail(SOCP_E_UNSUPPORTED, "librccl.so.1 not found");
  HIPCHK(hipSetDevice(ctx->device));
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  auto* c = new socp_comm();
  c->ctx = ctx;
  c->device = ctx->device;
  c->nranks = nranks;
  c->rank = rank;
  const ncclResult_t r = R->init_rank(&c->comm, nranks, u, rank);
  if (r != ncclSuccess) {
    delete c;
    return fail(SOCP_E_HIP, std::string("ncclCommInitRank: ") + R->err_str(r));
  }
  *out = c;
  return 0;
}

extern "C" int socp_comm_destroy(socp_comm* comm) {
  if (!comm) return 0;
  const Rccl* R = rccl();
  (void)hipSetDevice(comm->device);
  if (R && comm->comm) (void)R->destroy(comm->comm);
  comm->pairs.release();
  delete comm;
  return 0;
}

extern "C" int socp_allgather_status(socp_comm* comm, int64_t batch, const int32_t* status, const int32_t* iters,
                                     int32_t* out) {
  if (!comm) return fail(SOCP_E_INVALID, "comm is NULL");
  if (batch < 0) return fail(SOCP_E_INVALID, "negative batch");
  if (batch == 0) return 0;
  if (!status || !iters || !out) return fail(SOCP_E_INVALID, "NULL pointer");
  const Rccl* R = rccl();
  socp_ctx* ctx = comm->ctx;
  HIPCHK(hipSetDevice(ctx->device));
  if (comm->pairs.ensure((size_t)batch * 2 * sizeof(int32_t))) return fail(SOCP_E_NOMEM, "device allocation failed");
  int32_t* pairs = (int32_t*)comm->pairs.p;
  hipLaunchKernelGGL(socp_pair_kernel, dim3((unsigned)((batch + 255) / 256)), dim3(256), 0, ctx->stream, batch,
                     status, iters, pairs);
  HIPCHK(hipGetLastError());
  RCCLCHK(R, R->all_gather(pairs, out, (size_t)batch * 2, ncclInt32, comm->comm, ctx->stream));
  return 0;
}

extern "C" int socp_allgather_outcomes(socp_comm* comm, int64_t batch, const int32_t* status, const int32_t* iters,
                                       const double* res, socp_outcome* out) {
  if (!comm) return fail(SOCP_E_INVALID, "comm is NULL");
  if (batch < 0) return fail(SOCP_E_INVALID, "negative batch");
  if (batch == 0) return 0;
  if (!status || !iters || !out) return fail(SOCP_E_INVALID, "NULL pointer");
  const Rccl* R = rccl();
  socp_ctx* ctx = comm->ctx;
  HIPCHK(hipSetDevice(ctx->device));
  if (comm->pairs.ensure((size_t)batch * sizeof(socp_outcome))) return fail(SOCP_E_NOMEM, "device allocation failed");
  socp_outcome* rec = (socp_outcome*)comm->pairs.p;
  hipLaunchKernelGGL(socp_outcome_kernel, dim3((unsigned)((batch + 255) / 256)), dim3(256), 0, ctx->stream, batch,
                     status, iters, res, rec);
  HIPCHK(hipGetLastError());
  // records travel as raw bytes: 32 B each, one ring all-gather over xGMI
  RCCLCHK(R, R->all_gather(rec, out, (size_t)batch * sizeof(socp_outcome), ncclUint8, comm->comm, ctx->stream));
  return 0;
}
