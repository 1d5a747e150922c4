/*
 * gll.h -- C ABI of the MI355X (gfx950) Graph Learning Layer hot path.
 *
 * Drop-in boundary for `LaplaceLearningSparseHard.apply(X, label_matrix, tau, epsilon)`
 * of jwcalder/GraphLearningLayer.  Each entry point names the reference interface it
 * replaces (file:line in the reference snapshot).  Plain pointers and sizes only: device
 * pointers are HIP device memory, `stream` is a hipStream_t passed as void*.  Row-major,
 * fp32 features, int32 indices.  Inputs and outputs are caller-owned; the caller also owns
 * one workspace block per call (size from gll_workspace_bytes) that carries the graph from
 * gll_forward to gll_backward (the reference keeps the same state on `ctx`,
 * GLL.py:69-70).  Nothing here synchronises the host; nothing allocates; every call is
 * stream-ordered and reentrant per stream.  Return codes: 0 ok, < 0 error (no exceptions
 * cross the ABI).
 */
#ifndef GLL_H
#define GLL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GLL_OK 0
#define GLL_ERR_INVALID_ARG (-1)
#define GLL_ERR_UNSUPPORTED (-2)
#define GLL_ERR_HIP (-3)

/* dtype codes of label_matrix / grad_output (the reference accepts float32 and int64
 * one-hot label matrices: FullySup.py:153, train_and_adversarial.py:712) */
#define GLL_DT_F32 0
#define GLL_DT_F64 1
#define GLL_DT_I64 2

/* status words the device writes into the workspace (read with gll_status_offset) */
#define GLL_ST_TINY_EPS 0      /* eps_i < 1e-10 seen (GLL.py:240-241 warns) */
#define GLL_ST_FWD_NONCONV 1   /* forward CG columns that hit max_iter */
#define GLL_ST_FWD_ITERS 2     /* max forward CG iterations over columns */
#define GLL_ST_BWD_NONCONV 3   /* adjoint CG columns that hit max_iter */
#define GLL_ST_BWD_ITERS 4     /* max adjoint CG iterations over columns */
#define GLL_ST_KNN_RESCAN 5    /* kNN rows whose candidate set failed the Gram error certificate
                                * and were re-ranked exactly over every column under the bound
                                * (diagnostic count; the result is exact either way) */
#define GLL_ST_SOLVE_FAILED 6  /* nonzero: the fused backward's gradient workgroups gave up
                                * waiting for the adjoint solves (1 s of wall clock); the gradient was written
                                * as NaN.  The Python layer raises RuntimeError on it */
#define GLL_ST_KNN_MERGE 7     /* kNN rows with more than 64 columns at the threshold scan's
                                * bound (ties): the full-row fallback ran (diagnostic count) */
                               /* (words 8, 9, 11 are internal) */
#define GLL_ST_GRID_RESCUED 10 /* whole-GPU CG solves whose grid barrier timed out (a workgroup
                                * was not resident: other kernels held the CUs) and that one
                                * workgroup then solved alone -- correct, slower (count) */
#define GLL_ST_NWORDS 16

/* gll_problem.flags: code-path choices for tests and A/B runs; none changes a result beyond
 * fp32 summation order (each is compared against the default path in tests/) */
#define GLL_FLAG_CG_GRID 1      /* solve Luu with the whole-GPU CG even for small m */
#define GLL_FLAG_CG_PERCOL 8    /* single graphs with m > 2048: per-column CG instead of the whole-GPU CG */
#define GLL_FLAG_DIAG_GRID_OVERSUB 128 /* tests: size the whole-GPU CG at one row per workgroup,
                                        * far past its co-resident capacity -- the launch must
                                        * be refused */
#define GLL_FLAG_DIAG_GRID_FAIL 256    /* tests: inject a grid-barrier failure into the
                                        * whole-GPU CG (the rescue solve takes over) */
#define GLL_FLAG_CG_ELL 512     /* per-column CG: register-ELL kernel even where the balanced
                                 * (virtual-row) kernel would run */
#define GLL_FLAG_CG_VR 1024     /* per-column CG: balanced (virtual-row) kernel wherever it can
                                 * run (m <= 2048) */
#define GLL_FLAG_GRAD_ROWS 2048 /* feature gradient: whole-row kernel even where the
                                 * feature-chunked one would run */
#define GLL_FLAG_GRAD_CHUNK 4096 /* feature gradient: feature-chunked kernel wherever it can
                                  * run (d >= 128, d % 4 == 0) */
#define GLL_FLAG_GRAM_INLINE 8192 /* 128-tile Gram: split each tile's rows inline instead of
                                   * pre-split planes + LDS-DMA */
#define GLL_FLAG_BWD_UNFUSED 16384 /* single small graphs, fixed eps: adjoint CG and feature
                                    * gradient as two launches instead of the fused one */
#define GLL_FLAG_KNN_PANEL 65536   /* single graphs: build the kNN in row panels of 1,024 rows
                                    * (an O(panel x n) distance buffer instead of n x n; automatic
                                    * past 32 GiB of n x n distances, panels of 8 GiB) */
#define GLL_FLAG_D2_F32 131072     /* pre-split Gram route (batches): keep the distance matrix
                                    * fp32 instead of fp16 x 2^e */
#define GLL_FLAG_ROW_ORDER_OFF 262144 /* large single graphs: process the kNN select and the
                                       * chunked gradient in row-index order instead of the
                                       * pivot-grouped locality order (A/B; results identical) */
#define GLL_FLAG_ALL (1 | 8 | 128 | 256 | 512 | 1024 | 2048 | 4096 | 8192 | 16384 | 65536 | \
                      131072 | 262144)
/* (Retired, rejected with GLL_ERR_INVALID_ARG: 2 GRAM_NARROW, 4 CG_CLASSIC, 16 GRAM_F32,
 * 32 CG_PIPE, 64 GRAM_NOSPLIT, 32768 CG_PAIRS -- variants that lost their A/B runs.) */

/* Process-wide test knobs (gll_set_knob): each forces a code path that the automatic choice
 * would not take on the test's shape; 0 = automatic.  None changes a result. */
#define GLL_KNOB_VR_RV 0      /* balanced CG: virtual rows per thread (4 / 8 / 10) */
#define GLL_KNOB_GRID_CAP 1   /* whole-GPU CG: co-resident workgroup capacity */
#define GLL_KNOB_GRAM_TILE 2  /* pre-split Gram: 128- or 256-row tiles */
#define GLL_KNOB_SEL_FORM 3   /* kNN select form: 1 latency (PG 2), 2 occupancy (knn.hip) */
#define GLL_KNOB_GRAM_TAIL 4  /* 256-tile Gram's short last round: 1 none, 2 as 128-subtiles
                               * instead of 64-subtiles (knn.hip) */
#define GLL_KNOB_ROW_PRE 5    /* row build label prefetch: 1 on, 2 off (rows.hip) */
#define GLL_KNOB_COUNT 6
int gll_set_knob(int knob, int value);

typedef struct gll_problem {
    int32_t n;        /* rows of X = base + m; labeled rows first (GLL.py:11,32) */
    int32_t d;        /* feature dimension */
    int32_t base;     /* labeled rows = label_matrix.shape[0] (GLL.py:32) */
    int32_t C;        /* classes = label_matrix.shape[1] */
    int32_t K;        /* neighbours incl. self, 2 <= K <= 257 (K >= n is clamped to n); the reference
                       * hard-codes 25 (GLL.py:27) */
    int32_t max_iter; /* CG iteration cap per column; 0 => 1000 */
    float tau;        /* diagonal regulariser of Luu (GLL.py:48) */
    float eps;        /* > 0: fixed epsilon (GLL.py:226); <= 0: 'auto' (GLL.py:200-205) */
    float rtol;       /* CG stop: ||r_c|| <= rtol ||b_c|| per column; 0 => 1e-6 */
    int32_t flags;    /* GLL_FLAG_* bits, 0 by default */
    int32_t* status_sink; /* optional device words (GLL_ST_NWORDS): when non-NULL the public
                           * status words accumulate there across calls (sticky; the caller
                           * reads and clears them when it likes) instead of the workspace.
                           * Batched calls: GLL_ST_FWD_ITERS / BWD_ITERS in a sink hold the
                           * iterations of graph 0 and of every column that hit max_iter --
                           * not of every column workgroup of the batch, which would all
                           * update one word (B = 64 NS: 640 same-address atomics per CG
                           * launch, ~4 us) */
} gll_problem;

/* Bytes of device workspace one forward+backward pair needs. */
size_t gll_workspace_bytes(const gll_problem* p);

/* Replaces LaplaceLearningSparseHard.forward (GLL.py:14-73) incl. knn_sym_dist
 * (GLL.py:180-244), csgraph.laplacian (GLL.py:29) and the spsolve of GLL.py:53.
 * X: n x d fp32 (16-B aligned for the vector path), Y: base x C of y_dtype,
 * U: m x C float64 output (the reference returns float64, GLL.py:66). */
int gll_forward(const gll_problem* p, const float* X, const void* Y, int y_dtype,
                void* workspace, double* U, void* stream);

/* Replaces LaplaceLearningSparseHard.backward (GLL.py:76-177): adjoint solve (GLL.py:93),
 * edge gradient loop (GLL.py:111-120), auto-eps term (GLL.py:124-139) and the Laplacian
 * SpMM (GLL.py:146-159).  gbar: m x C of g_dtype; gradX: n x d fp32 output.
 * `workspace` must be the block the matching gll_forward filled. */
int gll_backward(const gll_problem* p, const float* X, const void* Y, int y_dtype,
                 void* workspace, const void* gbar, int g_dtype, float* gradX, void* stream);

/* Batched variants (no reference counterpart -- B independent calls of
 * GLL.py:14-177 on graphs of one shape, e.g. the 6 PGD calls of one minibatch in
 * train_and_adversarial.py:711-749, or one minibatch per rank-local stream).  Graph g reads
 * X + g*n*d, Y + g*base*C and writes U + g*m*C (gbar + g*m*C, gradX + g*n*d in the
 * backward); `workspace` holds B consecutive blocks of gll_workspace_bytes(p) bytes.  Each
 * kernel is launched once for all B graphs (grid.y = graph), so small graphs fill the GPU.
 * Results are bitwise those of B single calls.  1 <= B <= 65535. */
int gll_forward_batched(const gll_problem* p, int B, const float* X, const void* Y, int y_dtype,
                        void* workspace, double* U, void* stream);
int gll_backward_batched(const gll_problem* p, int B, const float* X, void* workspace,
                         const void* gbar, int g_dtype, float* gradX, void* stream);

/* Graph only (the device half of knn_sym_dist, GLL.py:180-244): kNN search, symmetric
 * CSR, eps, weights and degrees into the workspace; no solve.  Requires p->base == 0
 * (no labeled block; size the workspace for that problem).  Read the arrays with
 * gll_workspace_view. */
int gll_graph(const gll_problem* p, const float* X, void* workspace, void* stream);

/* Device pointers of the arrays held in a workspace (for the host mirror and tests). */
typedef struct gll_view {
    int32_t* knn_idx;  /* n x K  neighbour indices, self first, ascending distance */
    float* knn_d2;     /* n x K  squared distances (fp32, exact difference form)    */
    float* eps;        /* n      epsilon_i                                           */
    int32_t* row_start; /* n     first entry of graph row i (symmetric kNN graph,   */
    int32_t* row_len;   /* n     no diagonal); entries row_start..+row_len          */
    int32_t* col;      /* E      column indices, ascending within a row             */
    float* w;          /* E      W_ij = exp(-4 d_ij^2 / (eps_i eps_j))               */
    float* d2;         /* E      d_ij^2                                              */
    float* deg;        /* n      weighted degree                                     */
    float* U32;        /* m x C  forward solution, fp32                              */
    float* wadj;       /* m x C  adjoint solution (after gll_backward)               */
    int32_t* status;   /* GLL_ST_NWORDS status words                                 */
} gll_view;
int gll_workspace_view(const gll_problem* p, void* workspace, gll_view* out);

/* Multi-RHS Jacobi-preconditioned CG on a general SPD CSR matrix (device replacement of
 * stable_conjgrad, GLL.py:247-276, as used by utils.laplace, utils.py:589).
 * A: m x m CSR (row_ptr m+1, col, val) fp32; b, x: m x C row-major fp32 (x is output).
 * Stops per column when ||r_c||_2 <= atol (absolute, like stable_conjgrad's tol) or
 * max_iter.  `iters` (device int, may be NULL) receives the max iteration count,
 * `nonconv` (device int, may be NULL) the columns that hit max_iter.  `workspace`
 * (gll_cg_csr_workspace_bytes) holds the Krylov vectors: required when m > 2048 (those
 * systems run on the whole GPU as one ordinary launch sized within the co-resident
 * workgroup capacity, C <= 16; a lost grid barrier is rescued by one workgroup solving
 * alone, counted in GLL_ST_GRID_RESCUED), may be NULL when 5 m floats fit in LDS. */
size_t gll_cg_csr_workspace_bytes(int m, int C);
int gll_cg_csr(int m, int C, const int32_t* row_ptr, const int32_t* col, const float* val,
               const float* b, float* x, float atol, int max_iter, int32_t* iters,
               int32_t* nonconv, void* workspace, void* stream);

/* Instrumentation for bench.py: with period p > 0, every p-th launch of kernel `kid` is
 * bracketed by HIP events on its stream (p = 0 disables); gll_prof_read synchronises those
 * events and returns the summed milliseconds and the number of bracketed launches, then
 * clears them. */
#define GLL_K_GRAM 0      /* gram_d2_kernel: squared distances on split-bf16 MFMA (x = hi + lo,
                           * three bf16 products; candidates only, the select re-ranks exactly) */
#define GLL_K_SELECT 1    /* knn_select_kernel: top-K + exact re-rank + reverse scatter */
#define GLL_K_FINALIZE 2  /* row_build_kernel: symmetric rows, W, degree, rhs */
#define GLL_K_CG 3        /* cg_*_kernel: Jacobi-CG solves (forward and adjoint) */
#define GLL_K_EDGE 4      /* edge_coef_kernel: auto-eps edge coefficients */
#define GLL_K_GRAD 5      /* grad_spmm_kernel: feature gradient */
#define GLL_K_BWD 6       /* cg_grad_fused_kernel: adjoint CG + feature gradient in one launch
                           * (single small graphs, fixed eps) */
#define GLL_K_COUNT 7
int gll_prof_enable(int kid, int period);
int gll_prof_read(int kid, double* ms_total, int* count);
const char* gll_kernel_name(int kid);

/* Build identity: sha256 (16 hex) of the sources, headers and flags this library was built
 * from (graphlearninglayer_amd/build.py source_digest).  bench.py cites only profiles
 * recorded against the same identity. */
const char* gll_build_id(void);

/* Human-readable message for a return code. */
const char* gll_strerror(int code);

#ifdef __cplusplus
}
#endif
#endif /* GLL_H */
