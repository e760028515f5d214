/*
 * socp.h — C ABI of libsocp, the MI355X-native batched dense SOCP solver.
 *
 * This is the drop-in boundary for the dense path of BenChung/Socp.jl.
 * The reference has no C ABI of its own: its plugin interface is Julia multiple
 * dispatch (abstract type KKTSolver{T}, Socp.jl:77-78) and the per-iteration
 * calls compute_scaling / setup_iter / solve_kkt made by solve_socp
 * (solver.jl:105-151).  Every entry point below names the reference interface
 * it replaces; INTEGRATION.md shows the `ccall` binding a Julia maintainer adds.
 *
 * Problem (reference Socp.jl:20-38, README.md:4):
 *     minimize c'x   s.t.  A x = b,   G x + s = h,   s in K
 * K is a product of cones listed POC-first then SOC, contiguous over 0..k-1
 * (scalings.jl:102).  All arithmetic is IEEE fp64.
 *
 * Layout (shared by host and device pointers):
 *   - one cone description for the whole batch (every problem has the same
 *     dims and cone structure, as the reference's Problem{C,n,m,k} type does);
 *   - per problem, matrices are dense COLUMN-MAJOR (Julia order):
 *       A: m x n  -> A[p*m*n + j*m + i] = A_p(i,j)
 *       G: k x n  -> G[p*k*n + j*k + i] = G_p(i,j)
 *     vectors are stacked batch-major: c[p*n + j], b[p*m + i], h[p*k + i], ...
 *
 * Errors: every function returns 0 on success and a negative SOCP_E* code on
 * an API error; socp_last_error() gives a message (thread-local).  Numerical
 * failures are NOT API errors: they are reported per problem in status[]
 * (the reference instead throws PosDefException / DomainError and aborts the
 * solve: densesolver.jl:47,51; Julia sqrt of a negative argument).
 */
#ifndef SOCP_H
#define SOCP_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return codes (API errors) ---- */
#define SOCP_OK 0
#define SOCP_E_INVALID (-1)     /* bad argument / shape (reference: AssertionError, Socp.jl:43-47) */
#define SOCP_E_UNSUPPORTED (-2) /* dims not covered by any compiled kernel                          */
#define SOCP_E_HIP (-3)         /* HIP runtime error                                                 */
#define SOCP_E_NOMEM (-4)       /* device allocation failed                                          */

/* ---- per-problem status (numerical outcome) ---- */
#define SOCP_CONVERGED 0      /* exit test ||rd||+||rp||+z's < tol met (solver.jl:122)               */
#define SOCP_MAXIT 1          /* iteration cap reached (solver.jl:105)                               */
#define SOCP_CHOL_H_FAILED 2  /* H = G'W^-2G (+A'A) not positive definite (densesolver.jl:47)        */
#define SOCP_CHOL_S_FAILED 3  /* S = A H^-1 A' not positive definite (densesolver.jl:51)            */
#define SOCP_DOMAIN_ERROR 4   /* sqrt of a negative number: Julia throws DomainError (scalings.jl:46,47,57,68,91; mats.jl:71) */

/* ---- cone kinds (reference Socp.jl:8-16) ---- */
#define SOCP_CONE_POC 0 /* nonnegative orthant, POC{D}(offs) */
#define SOCP_CONE_SOC 1 /* second-order cone,   SOC{D}(offs) */

typedef struct socp_dims {
  int64_t batch; /* number of independent problems B                    */
  int32_t n;     /* variables        (Problem.n, Socp.jl:36)             */
  int32_t m;     /* equality rows    (Problem.m)                         */
  int32_t k;     /* cone rows        (Problem.k)                         */
  int32_t ncones;
} socp_dims;

/* Solver constants.  Defaults (socp_params_default) equal the reference's
 * hard-coded values: maxit 40 (solver.jl:105), tol 1e-5 absolute (:122),
 * step 0.99 (:146), sigma exponent 3 (:133), init shift threshold 1e-10 (:91,97). */
typedef struct socp_params {
  int32_t maxit;
  int32_t sigma_exp;
  double tol;      /* tol = 0 gives the fixed-iteration ("fixed-K") mode        */
  double step;
  double init_eps;
  int32_t flags;   /* SOCP_F_* bit set */
  int32_t reserved;
} socp_params;

#define SOCP_F_DEVICE_PTRS 1 /* all data pointers are device (HBM) pointers */
#define SOCP_F_WARM_START 2  /* x,y,z,s hold the starting iterate: skip the init solve (solver.jl:68-104) */
#define SOCP_F_FORCE_LARGE 4 /* run the blocked kernel even where the register-resident one applies (testing, tuning) */
/* Form Li = H^-1 explicitly, as densesolver.jl:47-48 does (ldiv!(Li,
 * cholesky!(H), I): H = L L', then Li = L^-T L^-1 from the factor; S^-1 the
 * same way), and use it in every solve (:73,83) -- the reference's operation
 * order.  By
 * default the kernels factor H = L L' (cholesky!, :47) and replace every
 * product with Li by two triangular solves (A Li enters as Z = L^-1 A',
 * S = Z'Z): the same linear algebra in exact arithmetic, far more accurate
 * near the end of a solve -- where the explicit inverse decides convergence
 * (a pure LP: chol(H) fails on every problem with it, converges without; see
 * DESIGN.md §9).  Honoured by socp_batch_solve[_ex], socp_batch_kkt_solve,
 * socp_dense_create (for all calls of the handle) and socp_ingest_submit. */
#define SOCP_F_EXPLICIT_INVERSE 8

typedef struct socp_ctx socp_ctx;

/* Library / context.  One context per host thread, each owning a HIP stream
 * (the reference indexes CHOLMOD state by Threads.threadid(), cholutils.jl:73). */
const char* socp_last_error(void);
const char* socp_version(void);
void socp_params_default(socp_params* p);
int socp_ctx_create(int device, socp_ctx** out);
int socp_ctx_destroy(socp_ctx* ctx);
int socp_ctx_sync(socp_ctx* ctx);
/* hipStream_t of the context (as void*) so callers can order their own work. */
void* socp_ctx_stream(socp_ctx* ctx);
/* Make the context issue its work on the caller's hipStream_t (as void*), e.g.
 * torch.cuda.current_stream().cuda_stream, so the solve is ordered after the
 * caller's producers of its inputs and before their consumers.  NULL is HIP's
 * null (default) stream -- torch's default current stream.  socp_ctx_reset_stream
 * returns to the context's own stream.  Work already queued on the previous
 * stream stays ordered before later work (an event wait is inserted). */
int socp_ctx_set_stream(socp_ctx* ctx, void* stream);
int socp_ctx_reset_stream(socp_ctx* ctx);

/* 1 if a compiled kernel accepts the dims: the register-resident kernel (one
 * wavefront per problem, <= 8 cones, m <= 64; k <= 128 for n <= 48, k <= 96
 * for 48 < n <= 64: the compiled variant table, socp.jl_amd/csrc/gen_inst.py)
 * or the blocked kernel (n, m <= 2048, <= 64 cones, k <= 2^21 -- its
 * LDS / vector offsets are 32-bit; one 512-thread workgroup per problem), which
 * also takes every register-kernel shape.  The
 * blocked kernel keeps the problem's vectors in the 160 KiB LDS of a CU when
 * they fit (C4, n=512 m=64 k=640, uses 126 KiB) and in its HBM workspace slot
 * otherwise (e.g. k = 1000 at n = 512).  Other shapes return
 * SOCP_E_UNSUPPORTED from the solve entries.  Every entry rejects batch >
 * 2^31-1 (device problem indices are int32). */
int socp_supported(const socp_dims* dims);

/* Batched solve: replaces solve_socp(prob, SolverState(prob, DenseSolver(prob)))
 * (solver.jl:40-153 with the DenseSolver plugin, densesolver.jl:1-90), run once
 * per problem of the batch.
 *   cone_kind/offs/dim : ncones entries (POC first, then SOC), host pointers.
 *   c,A,b,G,h          : problem data (layout above).
 *   sing               : per-problem flag; 1 if cholesky(G'G) fails (Socp.jl:49-56).
 *                        NULL -> computed on device by the same positive-definiteness
 *                        test the kernel uses for H.
 *   x,y,z,s            : out (in as well with SOCP_F_WARM_START): final iterate
 *                        (the reference returns State(x,y,z,s), solver.jl:152).
 *   iters, status      : out, per problem (int32); iters = completed Newton steps.
 * With SOCP_F_DEVICE_PTRS the call is stream-ordered and returns without
 * synchronising; otherwise it copies, solves and synchronises.
 * Diagnostics: with SOCP_DUMP_DIR=<dir> in the environment, the first
 * SOCP_DUMP_COUNT (default 1) problems of every batch are written to
 * <dir>/problem<p>_{A,G,c,b,h,initv,cones}.txt, as the reference's commented
 * dumps do (solver.jl:48-67,75-82). */
int socp_batch_solve(socp_ctx* ctx, const socp_dims* dims,
                     const int32_t* cone_kind, const int32_t* cone_offs, const int32_t* cone_dim,
                     const double* c, const double* A, const double* b,
                     const double* G, const double* h, const uint8_t* sing,
                     const socp_params* params,
                     double* x, double* y, double* z, double* s,
                     int32_t* iters, int32_t* status);

/* Same, plus per-problem final residual norms: res[3*p+0]=||rd||, [1]=||rp||, [2]=z's
 * (the quantities of the exit test, solver.jl:109-122), evaluated at the returned iterate. */
int socp_batch_solve_ex(socp_ctx* ctx, const socp_dims* dims,
                        const int32_t* cone_kind, const int32_t* cone_offs, const int32_t* cone_dim,
                        const double* c, const double* A, const double* b,
                        const double* G, const double* h, const uint8_t* sing,
                        const socp_params* params,
                        double* x, double* y, double* z, double* s,
                        int32_t* iters, int32_t* status, double* res);

/* Single-problem plugin entries.  They replace the two KKTSolver methods of
 * DenseSolver so the reference's own KKT golden (runtests.jl:95-128) runs
 * through the HIP path:
 *   setup_iter(ss::DenseSolver, pr, state, scaling)   densesolver.jl:41-52
 *   solve_kkt (ss::DenseSolver, pr, state, scaling, dx,dy,dz,ds, cx,cy,cz,cs)   densesolver.jl:54-90
 * Here both happen in one device call on a batch: given the iterate (s,z) the
 * NT scaling is computed (scalings.jl:101-110), the KKT matrix factored, and the
 * system solved for the right-hand side (dx,dy,dz,ds) -> (cx,cy,cz,cs).
 * kkt_status[p]: 0 ok, SOCP_CHOL_H_FAILED, SOCP_CHOL_S_FAILED, SOCP_DOMAIN_ERROR. */
int socp_batch_kkt_solve(socp_ctx* ctx, const socp_dims* dims,
                         const int32_t* cone_kind, const int32_t* cone_offs, const int32_t* cone_dim,
                         const double* A, const double* G, const uint8_t* sing,
                         const double* s, const double* z,
                         const double* dx, const double* dy, const double* dz, const double* ds,
                         double* cx, double* cy, double* cz, double* cs,
                         int32_t* kkt_status, int32_t flags);  /* flags: SOCP_F_DEVICE_PTRS | SOCP_F_FORCE_LARGE */

/* The same two methods split the way the reference's KKTSolver plugin is
 * (densesolver.jl): a handle stands for a batch of DenseSolver objects.
 *   socp_dense_create      replaces DenseSolver(...) construction
 *                          (densesolver.jl:9-39): A and G (and sing, or NULL
 *                          for the cholesky(G'G) test at every setup) are
 *                          copied into the handle once;
 *   socp_dense_setup_iter  replaces setup_iter(ss, pr, state, scaling)
 *                          (densesolver.jl:41-52): NT scaling of (s, z), H and
 *                          its factorisation, kept on the device as one factor
 *                          record per problem.  By default the record holds
 *                          the Cholesky factor of H (register kernel, m <= 16:
 *                          16x16 tiles, L_PP^-1 on the diagonal; blocked
 *                          kernel: L in place, L_PP^-1 in the diagonal
 *                          blocks), Z = L^-1 A' and S^-1 for S = Z'Z =
 *                          A H^-1 A'; H^-1 itself is never formed.  Where m > 16
 *                          on the register kernel, or with
 *                          SOCP_F_EXPLICIT_INVERSE, it holds Li = H^-1, A Li
 *                          (or Li A') and S^-1, as densesolver.jl:48-51 do;
 *                          status[p]: 0, SOCP_CHOL_H_FAILED,
 *                          SOCP_CHOL_S_FAILED or SOCP_DOMAIN_ERROR (where the
 *                          reference throws PosDefException / DomainError);
 *   socp_dense_solve_kkt   replaces solve_kkt(ss, ...) (densesolver.jl:54-90)
 *                          against the last setup_iter; call it any number of
 *                          times (the solver calls it twice per iteration,
 *                          solver.jl:125-145).  status[p] = 0, or setup_iter's
 *                          status with NaN outputs for a problem whose setup
 *                          failed.
 * flags (at create, for all calls of the handle): SOCP_F_DEVICE_PTRS (every
 * pointer, A and G included, is a device pointer; the calls are then
 * stream-ordered on the context's stream and return without synchronising) |
 * SOCP_F_FORCE_LARGE.  With host pointers each setup_iter moves 2k doubles
 * per problem host-to-device and each solve_kkt n+m+2k; A and G move once, at
 * create (socp_dense_h2d_bytes reports the last call's count).  The results are
 * bitwise those of socp_batch_kkt_solve on the same inputs.  Device memory:
 * socp_dense_record_bytes() per problem plus A, G. */
typedef struct socp_dense socp_dense;
int socp_dense_create(socp_ctx* ctx, const socp_dims* dims,
                      const int32_t* cone_kind, const int32_t* cone_offs, const int32_t* cone_dim,
                      const double* A, const double* G, const uint8_t* sing, int32_t flags,
                      socp_dense** out);
int socp_dense_setup_iter(socp_dense* h, const double* s, const double* z, int32_t* status);
int socp_dense_solve_kkt(socp_dense* h, const double* dx, const double* dy, const double* dz,
                         const double* ds, double* cx, double* cy, double* cz, double* cs,
                         int32_t* status);
int socp_dense_h2d_bytes(const socp_dense* h, int64_t* bytes);
int64_t socp_dense_record_bytes(const socp_dense* h);
int socp_dense_destroy(socp_dense* h);

/* The rank-update plugin: SparseSolver with SqrScaling (spsolver.jl:1-130,
 * sqrscalings.jl:8-214), the solver the reference's own tests and MOI run.
 *   socp_sqr_create      replaces SparseSolver(pr) (spsolver.jl:24-57): A, G
 *                        and sing (the Problem's type parameter; NULL = no
 *                        problem is sing) copied into the handle once;
 *   socp_sqr_setup_iter  replaces compute_scaling(cones, ::SqrScaling, s, z)
 *                        (sqrscalings.jl:177-185) + setup_iter(::SparseSolver)
 *                        (spsolver.jl:60-84): W^-2 = D + uu' - vv' per SOC cone,
 *                        L L' = G'DG (+A'A when sing), one rank-1 update with
 *                        G'u and one downdate with G'v per SOC cone
 *                        (modify_factors!, sqrscalings.jl:160-194), and the
 *                        factor of S = (L^-1 A')'(L^-1 A'); status[p] as for
 *                        socp_dense_setup_iter (a downdate that loses positive
 *                        definiteness is SOCP_CHOL_H_FAILED);
 *   socp_sqr_solve_kkt   replaces solve_kkt(::SparseSolver) (spsolver.jl:86-130)
 *                        by triangular solves against the record;
 *   socp_sqr_factor      problem p's factor L of H after the modifications
 *                        (n x n, column-major, zeros above the diagonal): the
 *                        Gfact CHOLMOD factor of spsolver.jl:13 as a dense matrix;
 *   socp_sqr_scaling     the SqrScaling fields l, wbs, mu (B x k, B x k,
 *                        B x ncones) of the last setup_iter.
 * CHOLMOD's fill-reducing permutation and supernodal LDL' are replaced by a
 * dense factor: results agree with the reference to rounding, not bitwise.
 * Shapes: n, m <= 1024, k <= 4096, <= 64 cones, the problem's vectors
 * within 160 KiB of LDS (socp_sqr_supported): one wavefront per problem for
 * n, m <= 64, one 256-thread workgroup above -- its factors packed in LDS,
 * or in the per-problem record when they and a right-hand-side chunk exceed
 * the LDS (n, m beyond about 160).  Flags and
 * host/device pointer semantics as socp_dense_*. */
typedef struct socp_sqr socp_sqr;
int socp_sqr_supported(const socp_dims* dims);
int socp_sqr_create(socp_ctx* ctx, const socp_dims* dims,
                    const int32_t* cone_kind, const int32_t* cone_offs, const int32_t* cone_dim,
                    const double* A, const double* G, const uint8_t* sing, int32_t flags,
                    socp_sqr** out);
int socp_sqr_setup_iter(socp_sqr* h, const double* s, const double* z, int32_t* status);
int socp_sqr_solve_kkt(socp_sqr* h, const double* dx, const double* dy, const double* dz,
                       const double* ds, double* cx, double* cy, double* cz, double* cs,
                       int32_t* status);
int socp_sqr_factor(socp_sqr* h, int64_t problem, double* L);
int socp_sqr_scaling(socp_sqr* h, double* l, double* wbs, double* mu);
/* solve_socp(prob, SolverState(prob, SparseSolver(prob))) (solver.jl:40-153)
 * for the handle's whole batch -- the reference's own tested configuration
 * (runtests.jl:143-144, 188-189, 204-244) -- with this plugin's setup_iter /
 * solve_kkt: initial point (the KKT system with W = I and the cone shift,
 * solver.jl:68-104), then up to params->maxit iterations with the reference's
 * exit test, per-problem status and masking (problems that stop are skipped by
 * every later launch).  c (B x n), b (B x m), h (B x k) in; x, y, z, s, iters,
 * status, res (B x 3: ||rd||, ||rp||, z's at the returned iterate; may be
 * NULL) out.  params NULL: socp_params_default.  Host or device pointers as
 * the handle's flags.  Afterwards the records hold the last factorisation.
 * With tol > 0 the call synchronises its stream every 4 iterations to stop
 * launching once every problem has stopped (converged or failed); such a call
 * cannot be captured into a HIP graph.  With tol <= 0 (fixed iteration count)
 * it issues only stream-ordered work until the final copies.
 * The initial point factors G'G (+ A'A where sing) with W = I: `sing` must be
 * the flag Problem() computes (Socp.jl:49-56, cholesky(G'G) fails).  Where the
 * given flag disagrees and that factorisation fails, the problem stops with
 * status SOCP_CHOL_H_FAILED at iteration 0 -- the reference's sparse `\`
 * (solver.jl:84) would solve the full KKT system instead. */
int socp_sqr_solve_socp(socp_sqr* h, const double* c, const double* b, const double* hvec,
                        const socp_params* params, double* x, double* y, double* z, double* s,
                        int32_t* iters, int32_t* status, double* res);
int socp_sqr_h2d_bytes(const socp_sqr* h, int64_t* bytes);
int64_t socp_sqr_record_bytes(const socp_sqr* h);
int socp_sqr_destroy(socp_sqr* h);

/* Device-side deterministic generator of feasible synthetic problems
 * (SURVEY.md §8(d)): counter-based SplitMix64 keyed on the GLOBAL problem
 * index first_problem + p, so shards of a multi-GPU run reproduce the same
 * problems.  Output pointers are device pointers with the layout above. */
int socp_generate(socp_ctx* ctx, const socp_dims* dims,
                  const int32_t* cone_kind, const int32_t* cone_offs, const int32_t* cone_dim,
                  uint64_t seed, int64_t first_problem,
                  double* c, double* A, double* b, double* G, double* h);

/* Ingest: pack a batch of sparse matrices in Julia's
 * SparseMatrixCSC form -- the storage of Problem.A and Problem.G
 * (Socp.jl:25,29) -- into the dense column-major batch layout above, on the
 * device.  Every matrix is rows x cols.  Problem p's nonzeros are
 * nz_offs[p] .. nz_offs[p+1]-1 of rowval/nzval; its column pointer is
 * colptr[p*(cols+1) .. p*(cols+1)+cols] (relative to nz_offs[p]).  Indices are
 * int64 with index_base 1 (Julia, zero-copy) or 0.  All pointers are device
 * pointers; dense[p*rows*cols + j*rows + i] is written for every element
 * (zeros included).  Duplicate (i,j) entries are summed, as sparse() does.
 * Returns SOCP_E_INVALID (after synchronising) if any row index or column
 * pointer is out of range; nothing else is validated. */
int socp_pack_csc(socp_ctx* ctx, int64_t batch, int32_t rows, int32_t cols,
                  const int64_t* nz_offs, const int64_t* colptr, const int64_t* rowval,
                  const double* nzval, int32_t index_base, double* dense);

/* Pipelined ingest of host-resident batches: the
 * reference builds each Problem on the host (Socp.jl:20-60); here a stream of
 * host batches flows through two slots of pinned (hipHostMalloc) staging so
 * batch i+1's host-to-device copy -- and, in the CSC form, its packing --
 * runs on a copy stream while batch i solves on the context's stream, and
 * batch i's results drain to pinned memory on a third stream.
 *   socp_ingest_create(ctx, dims, cones..., flags, &ing): dims.batch is the
 *       largest batch one submit may carry (pinned + device space for two
 *       such batches is allocated here); flags: SOCP_F_FORCE_LARGE.
 *   socp_ingest_submit(ing, B, c, A, b, G, h, sing, params, &ticket): host
 *       arrays in the batch layout above, copied into the slot's pinned
 *       block (no copy for arrays already written at the pointers
 *       socp_ingest_next_inputs returns), then everything is asynchronous.
 *       params->flags other than the defaults are ignored (no warm start).
 *   socp_ingest_submit_csc(...): A and G as the SparseMatrixCSC arrays of
 *       socp_pack_csc (host pointers; nz_offs[B] - nz_offs[0] nonzeros each),
 *       packed on the device on the copy stream.
 *   socp_ingest_wait(ing, ticket, x, y, z, s, iters, status, res): blocks
 *       until that batch's results are on the host and copies them out (res
 *       may be NULL).  A CSC batch with bad indices returns SOCP_E_INVALID here.
 * At most two tickets are outstanding: a third submit before the oldest is
 * waited for returns SOCP_E_INVALID.  Results are bitwise those of
 * socp_batch_solve_ex on the same inputs. */
typedef struct socp_ingest socp_ingest;
int socp_ingest_create(socp_ctx* ctx, const socp_dims* dims,
                       const int32_t* cone_kind, const int32_t* cone_offs, const int32_t* cone_dim,
                       int32_t flags, socp_ingest** out);
int socp_ingest_next_inputs(socp_ingest* ing, double** c, double** A, double** b, double** G,
                            double** h, uint8_t** sing);
int socp_ingest_submit(socp_ingest* ing, int64_t batch, const double* c, const double* A,
                       const double* b, const double* G, const double* h, const uint8_t* sing,
                       const socp_params* params, int64_t* ticket);
int socp_ingest_submit_csc(socp_ingest* ing, int64_t batch, const double* c, const double* b,
                           const double* h, const uint8_t* sing,
                           const int64_t* A_nz_offs, const int64_t* A_colptr, const int64_t* A_rowval,
                           const double* A_nzval,
                           const int64_t* G_nz_offs, const int64_t* G_colptr, const int64_t* G_rowval,
                           const double* G_nzval, int32_t index_base, const socp_params* params,
                           int64_t* ticket);
int socp_ingest_wait(socp_ingest* ing, int64_t ticket, double* x, double* y, double* z, double* s,
                     int32_t* iters, int32_t* status, double* res);
int socp_ingest_destroy(socp_ingest* ing);

/* Multi-GPU outcome gather: problems shard across ranks
 * (one process per GPU) with no data-path exchange; the only collective is the
 * all-gather of each problem's (status, iters) over RCCL (xGMI between the
 * GPUs of a node).  This replaces nothing in the reference (which solves one
 * problem per call, solver.jl:40); it is the exchange step of the batched
 * multi-GPU drop-in.  RCCL (librccl.so.1) is opened on first use, so the rest
 * of the library has no RCCL dependency.
 *   rank 0: socp_comm_unique_id(id), then hands the 128 bytes to every rank
 *           (MPI broadcast, a file, torch.distributed ...);
 *   every rank: socp_comm_init(ctx, nranks, rank, id, &comm);
 *   socp_allgather_status(comm, B, status, iters, out): device pointers;
 *           out[(r*B + p)*2 + 0] = status, [.. + 1] = iters of rank r's
 *           problem p; equal B on every rank; stream-ordered on the
 *           context's stream (socp_ctx_sync to wait). */
#define SOCP_COMM_ID_BYTES 128
typedef struct socp_comm socp_comm;
int socp_comm_unique_id(unsigned char* id);
int socp_comm_init(socp_ctx* ctx, int nranks, int rank, const unsigned char* id, socp_comm** out);
int socp_comm_destroy(socp_comm* comm);
int socp_allgather_status(socp_comm* comm, int64_t batch, const int32_t* status, const int32_t* iters,
                          int32_t* out);
/* The SURVEY.md §8(e) record: per problem 32 bytes -- status, iters and the
 * exit-test quantities ||rd||, ||rp||, z's at the returned iterate
 * (solver.jl:109-122; res[] of socp_batch_solve_ex, NaN where res is NULL).
 * out[r*B + p] is rank r's problem p; device pointers; stream-ordered.  A comm
 * must be destroyed before the context it was created on. */
typedef struct socp_outcome {
  int32_t status;
  int32_t iters;
  double res_dual;   /* ||A'y + G'z + c|| */
  double res_primal; /* ||Ax - b||        */
  double gap;        /* z's               */
} socp_outcome;
int socp_allgather_outcomes(socp_comm* comm, int64_t batch, const int32_t* status, const int32_t* iters,
                            const double* res, socp_outcome* out);

/* Timing of the last solve's main kernel, measured with HIP events on the
 * context's stream (milliseconds), and its name.  socp_last_kernel_ms waits
 * for that launch. */
int socp_last_kernel_ms(socp_ctx* ctx, float* ms);
const char* socp_last_kernel_name(socp_ctx* ctx);
/* The main-kernel times of the context's last min(n, 64) timed launches,
 * oldest first, into ms[]; returns how many were written (< 0: error).  Each
 * launch records its own event pair, so a run of launches is timed without a
 * host synchronisation between them (bench.py's timed steps); the call waits
 * for the newest one. */
int socp_kernel_times(socp_ctx* ctx, float* ms, int n);

/* Testing hook (not part of the reference surface; diagnostic build
 * libsocp_diag.so only): when set to a device buffer of
 * batch*(2n^2+2k+nm+m^2) doubles, socp_batch_kkt_solve on the register kernel
 * dumps per problem the KKT matrix H = G'W^-2G (+A'A) (densesolver.jl:43-46),
 * its inverse Li (:48), lambda and wbar (scalings.jl:1-20), Li A' and S --
 * on the explicit-inverse path only (m > 16, or SOCP_F_EXPLICIT_INVERSE): the
 * default Cholesky path never forms Li and dumps nothing.  NULL disables. */
int socp_debug_set_kkt_dump(double* dev_buf);

/* Diagnostic hook: device buffer of 13 uint64 counters; in the phase-stamp build
 * (libsocp_stamps.so, -DSOCP_STAMPS) every solve adds per-phase shader-clock
 * cycles (load, scaling, residuals, U, SYRK, sweep(H), Schur, solve, step, init,
 * store, other) and the executed iterations.  The product build ignores it. */
int socp_debug_set_stamps(unsigned long long* dev_buf);

#ifdef __cplusplus
}
#endif
#endif /* SOCP_H */
