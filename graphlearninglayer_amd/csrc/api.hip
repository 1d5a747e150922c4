// api.hip -- the extern "C" boundary declared in include/gll.h.
//
// Orchestrates the kernels of knn.hip, rows.hip, solve.hip / gridcg.hip and grad.hip on the caller's
// stream.  No allocation, no host synchronisation: the caller owns the workspace (the
// Python mirror takes it from torch's caching allocator) and keeps it alive from
// gll_forward to gll_backward, as the reference keeps its graph on ctx (GLL.py:69-70).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "gll_internal.h"

namespace gll {

// ---------------------------------------------------------------------------------------
// Instrumentation: optional HIP event brackets around selected kernels (bench.py uses
// them to time the dominant kernel inside its timed region).
// ---------------------------------------------------------------------------------------
struct ProfState {
    int period[GLL_K_COUNT] = {};     // 0 = off, p = bracket every p-th launch
    long count[GLL_K_COUNT] = {};
    bool on[GLL_K_COUNT] = {};
    std::vector<hipEvent_t> pending[GLL_K_COUNT];  // start, stop, start, stop, ...
    std::vector<hipEvent_t> pool;
    std::mutex mu;
    hipEvent_t get() {
        if (!pool.empty()) {
            hipEvent_t e = pool.back();
            pool.pop_back();
            return e;
        }
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        return e;
    }
};
static ProfState g_prof;

thread_local ArmedLaunch g_armed;

// prof_begin arms a (start, stop) pair for the next launch_k on this thread; the dispatch
// packet records both, so the pair brackets exactly the first kernel of the region.
void prof_begin(int kid, hipStream_t) {
    if (!g_prof.on[kid]) return;
    std::lock_guard<std::mutex> lk(g_prof.mu);
    if ((g_prof.count[kid]++ % g_prof.period[kid]) != 0) return;
    hipEvent_t e0 = g_prof.get();
    hipEvent_t e1 = e0 ? g_prof.get() : nullptr;
    if (!e1) {
        if (e0) g_prof.pool.push_back(e0);
        return;
    }
    g_prof.pending[kid].push_back(e0);
    g_prof.pending[kid].push_back(e1);
    g_armed = ArmedLaunch{kid, e0, e1};
}

// A pair still armed at the end of the region was never consumed by a launch: drop it.
void prof_end(int kid, hipStream_t) {
    if (g_armed.kid != kid) return;
    std::lock_guard<std::mutex> lk(g_prof.mu);
    auto& v = g_prof.pending[kid];
    if (v.size() >= 2 && v.back() == g_armed.e1) {
        for (int i = 0; i < 2; ++i) {
            g_prof.pool.push_back(v.back());
            v.pop_back();
        }
    }
    g_armed = ArmedLaunch{};
}

bool debug_log() {
    static const bool dbg = getenv("GLL_DEBUG") != nullptr;
    return dbg;
}

hipError_t launch_status(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess && debug_log()) fprintf(stderr, "gll: %s: %s\n", what, hipGetErrorString(e));
    return e;
}

// ---------------------------------------------------------------------------------------
// Test knobs and cached device facts (gll_internal.h)
// ---------------------------------------------------------------------------------------
static std::atomic<int> g_knobs[GLL_KNOB_COUNT];

int knob(int id) { return g_knobs[id].load(std::memory_order_relaxed); }

static constexpr int kMaxDev = 64;
static std::atomic<int> g_cus[kMaxDev];

int device_cus() {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= kMaxDev) dev = 0;
    int v = g_cus[dev].load(std::memory_order_relaxed);
    if (v <= 0) {
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            v = 0;
        (void)hipGetLastError();
        v = v > 0 ? v : 1;
        g_cus[dev].store(v, std::memory_order_relaxed);
    }
    return v;
}

namespace {
struct OccKey {
    const void* fn;
    int nt;
    size_t lds;
    bool operator==(const OccKey& o) const { return fn == o.fn && nt == o.nt && lds == o.lds; }
};
struct OccHash {
    size_t operator()(const OccKey& k) const {
        return std::hash<const void*>()(k.fn) ^ (size_t(k.nt) << 20) ^ (k.lds * 0x9E3779B97F4A7C15ull);
    }
};
std::mutex g_occ_mu;
std::unordered_map<OccKey, int, OccHash> g_occ;
std::unordered_map<const void*, size_t> g_slds;
}  // namespace

// (one device model per process: MI355X nodes are homogeneous)
int occupancy_blocks(const void* fn, int nt, size_t lds) {
    std::lock_guard<std::mutex> lk(g_occ_mu);
    const OccKey key{fn, nt, lds};
    auto it = g_occ.find(key);
    if (it != g_occ.end()) return it->second;
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, nt, lds) != hipSuccess) nb = 0;
    (void)hipGetLastError();
    g_occ.emplace(key, nb);
    return nb;
}

size_t static_lds_bytes(const void* fn) {
    std::lock_guard<std::mutex> lk(g_occ_mu);
    auto it = g_slds.find(fn);
    if (it != g_slds.end()) return it->second;
    hipFuncAttributes at{};
    size_t stat = 8192;
    if (hipFuncGetAttributes(&at, fn) == hipSuccess) stat = at.sharedSizeBytes;
    (void)hipGetLastError();
    g_slds.emplace(fn, stat);
    return stat;
}

static const char* kKernelNames[GLL_K_COUNT] = {
    "gram_d2_kernel", "knn_select_kernel", "row_build_kernel",
    "cg_kernel",      "edge_coef_kernel",  "grad_spmm_kernel", "cg_grad_fused_kernel"};

static bool vec_ok(const float* X, int d) {
    return (d % 4 == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
}

static int check(const gll_problem* p) {
    if (!p) return GLL_ERR_INVALID_ARG;
    if (p->n < 2 || p->d < 1 || p->C < 1 || p->K < 2) return GLL_ERR_INVALID_ARG;
    if (p->base < 0 || p->base > p->n) return GLL_ERR_INVALID_ARG;
    const int K = p->K < p->n ? p->K : p->n;
    if (K - 1 > kMaxKm1Huge) return GLL_ERR_UNSUPPORTED;  // the wide select's LDS lists
    if (p->flags & ~GLL_FLAG_ALL) return GLL_ERR_INVALID_ARG;   // unknown (or retired) flags
    if (p->C > 256) return GLL_ERR_UNSUPPORTED;       // rhs accumulators per lane
    if ((p->d + 255) / 256 > 16) return GLL_ERR_UNSUPPORTED;  // d <= 4096 in the SpMM
    if (int64_t(p->n) * K > INT32_MAX / 2) return GLL_ERR_UNSUPPORTED;
    return GLL_OK;
}

static int hip_status(hipError_t e) { return e == hipSuccess ? GLL_OK : GLL_ERR_HIP; }

// Status words the caller reads: the sticky sink when given, else the workspace block.
static int32_t* public_status(const gll_problem* p, const Layout& L, void* ws) {
    return p->status_sink ? p->status_sink : L.at<int32_t>(ws, L.status);
}

static size_t dtype_size(int dt) { return dt == GLL_DT_F32 ? 4 : 8; }

// Strides of B contiguous problems: workspace blocks of L.total bytes, X / Y / U / gbar /
// gradX packed graph after graph; status words shared when they go to a sink.
static Batch make_batch(const gll_problem* p, const Layout& L, int B, int y_dtype, int g_dtype) {
    Batch bt;
    bt.B = B;
    bt.ws = L.total;
    bt.x = size_t(L.n) * L.d * sizeof(float);
    bt.y = size_t(L.base) * L.C * dtype_size(y_dtype);
    bt.u = size_t(L.m) * L.C * sizeof(double);
    bt.g = size_t(L.m) * L.C * dtype_size(g_dtype);
    bt.gx = bt.x;
    bt.st = p->status_sink ? 0 : L.total;
    return bt;
}

// kNN graph: gram (MFMA) -> select (+ reverse scatter) -> row build (+ weights, rhs)
static int build_graph(const gll_problem* p, const Layout& L, const Batch& bt, const float* X,
                       const void* Y, int y_dtype, void* ws, hipStream_t s) {
    const bool vec = vec_ok(X, p->d);
    const bool auto_eps = !(p->eps > 0.f);
    if (L.PR < L.n) {
        // row panels (Layout::PR < n: the n x n distances would not fit, or GLL_FLAG_KNN_PANEL):
        // each panel's rows against every column, then their selection; the reverse lists and
        // status counters accumulate across panels (reset by the first panel's Gram)
        if (bt.B > 1) return GLL_ERR_UNSUPPORTED;
        for (int r0 = 0; r0 < L.n; r0 += L.PR) {
            const int rows = L.n - r0 < L.PR ? L.n - r0 : L.PR;
            if (launch_gram_panel(L, ws, X, vec, r0, rows, s) != hipSuccess) return GLL_ERR_HIP;
            if (launch_select(L, bt, ws, X, p->eps, auto_eps, vec, public_status(p, L, ws), s,
                              r0, rows) != hipSuccess)
                return GLL_ERR_HIP;
        }
    } else {
        if (launch_gram(L, bt, ws, X, vec, s) != hipSuccess) return GLL_ERR_HIP;
        if (locality_order(L, bt) && launch_order(L, ws, s) != hipSuccess) return GLL_ERR_HIP;
        if (launch_select(L, bt, ws, X, p->eps, auto_eps, vec, public_status(p, L, ws), s) !=
            hipSuccess)
            return GLL_ERR_HIP;
    }
    return hip_status(launch_finalize(L, bt, ws, Y, y_dtype, p->tau, auto_eps ? 0.f : p->eps, s));
}

static int forward_impl(const gll_problem* p, int B, const float* X, const void* Y, int y_dtype,
                        void* ws, double* U, void* stream) {
    int rc = check(p);
    if (rc != GLL_OK) return rc;
    if (B < 1 || B > 65535) return GLL_ERR_INVALID_ARG;
    if (!X || !ws || (p->base > 0 && !Y) || (p->n > p->base && !U)) return GLL_ERR_INVALID_ARG;
    if (y_dtype != GLL_DT_F32 && y_dtype != GLL_DT_F64 && y_dtype != GLL_DT_I64)
        return GLL_ERR_INVALID_ARG;
    Layout L(*p);
    const Batch bt = make_batch(p, L, B, y_dtype, GLL_DT_F32);
    hipStream_t s = static_cast<hipStream_t>(stream);
    rc = build_graph(p, L, bt, X, Y, y_dtype, ws, s);
    if (rc != GLL_OK) return rc;
    const float rtol = p->rtol > 0.f ? p->rtol : 1e-6f;
    const int max_iter = p->max_iter > 0 ? p->max_iter : 1000;
    int32_t* st = public_status(p, L, ws);
    float* U32 = L.at<float>(ws, L.P) + size_t(L.base) * L.C;
    return hip_status(launch_cg_luu(L, bt, ws, L.at<float>(ws, L.rhs), bt.ws, GLL_DT_F32, U, U32,
                                    rtol, max_iter, st + GLL_ST_FWD_NONCONV,
                                    st + GLL_ST_FWD_ITERS, st + GLL_ST_SOLVE_FAILED, s));
}

static int backward_impl(const gll_problem* p, int B, const float* X, void* ws,
                         const void* gbar, int g_dtype, float* gradX, void* stream) {
    int rc = check(p);
    if (rc != GLL_OK) return rc;
    if (B < 1 || B > 65535) return GLL_ERR_INVALID_ARG;
    if (!X || !ws || !gradX || (p->n > p->base && !gbar)) return GLL_ERR_INVALID_ARG;
    if (g_dtype != GLL_DT_F32 && g_dtype != GLL_DT_F64) return GLL_ERR_INVALID_ARG;
    Layout L(*p);
    const Batch bt = make_batch(p, L, B, GLL_DT_F32, g_dtype);
    hipStream_t s = static_cast<hipStream_t>(stream);
    const float rtol = p->rtol > 0.f ? p->rtol : 1e-6f;
    const int max_iter = p->max_iter > 0 ? p->max_iter : 1000;
    int32_t* st = public_status(p, L, ws);
    float* wU = L.at<float>(ws, L.Wadj) + size_t(L.base) * L.C;
    const bool auto_eps = !(p->eps > 0.f);
    if (B == 1 && !auto_eps) {   // one small graph: adjoint CG + gradient in one launch
        const hipError_t e = launch_cg_grad_fused(L, ws, gbar, g_dtype, X, p->eps, gradX, rtol,
                                                  max_iter, st + GLL_ST_BWD_NONCONV,
                                                  st + GLL_ST_BWD_ITERS, st + GLL_ST_SOLVE_FAILED,
                                                  vec_ok(X, p->d), s);
        if (e != hipErrorNotSupported) return hip_status(e);
    }
    // adjoint solve: Luu is symmetric, so Luu^-T gbar = Luu^-1 gbar (GLL.py:93)
    hipError_t e = launch_cg_luu(L, bt, ws, gbar, bt.g, g_dtype, nullptr, wU, rtol, max_iter,
                                 st + GLL_ST_BWD_NONCONV, st + GLL_ST_BWD_ITERS,
                                 st + GLL_ST_SOLVE_FAILED, s);
    if (e != hipSuccess) return GLL_ERR_HIP;
    return hip_status(launch_backward_grad(L, bt, ws, X, auto_eps, p->eps, gradX,
                                           vec_ok(X, p->d), s));
}

}  // namespace gll

using namespace gll;

extern "C" {

size_t gll_workspace_bytes(const gll_problem* p) {
    if (check(p) != GLL_OK) return 0;
    return Layout(*p).total;
}

int gll_graph(const gll_problem* p, const float* X, void* ws, void* stream) {
    int rc = check(p);
    if (rc != GLL_OK) return rc;
    if (!X || !ws) return GLL_ERR_INVALID_ARG;
    if (p->base != 0) return GLL_ERR_INVALID_ARG;  // graph only: no labeled block
    Layout L(*p);
    // base = 0: every row is "unlabeled", rhs = 0 and no label is read
    return build_graph(p, L, make_batch(p, L, 1, GLL_DT_F32, GLL_DT_F32), X, nullptr, GLL_DT_F32,
                       ws, static_cast<hipStream_t>(stream));
}

int gll_forward(const gll_problem* p, const float* X, const void* Y, int y_dtype, void* ws,
                double* U, void* stream) {
    return forward_impl(p, 1, X, Y, y_dtype, ws, U, stream);
}

int gll_backward(const gll_problem* p, const float* X, const void* Y, int y_dtype, void* ws,
                 const void* gbar, int g_dtype, float* gradX, void* stream) {
    (void)Y;
    (void)y_dtype;
    return backward_impl(p, 1, X, ws, gbar, g_dtype, gradX, stream);
}

int gll_forward_batched(const gll_problem* p, int B, const float* X, const void* Y, int y_dtype,
                        void* ws, double* U, void* stream) {
    return forward_impl(p, B, X, Y, y_dtype, ws, U, stream);
}

int gll_backward_batched(const gll_problem* p, int B, const float* X, void* ws, const void* gbar,
                         int g_dtype, float* gradX, void* stream) {
    return backward_impl(p, B, X, ws, gbar, g_dtype, gradX, stream);
}

int gll_workspace_view(const gll_problem* p, void* ws, gll_view* out) {
    int rc = check(p);
    if (rc != GLL_OK) return rc;
    if (!ws || !out) return GLL_ERR_INVALID_ARG;
    Layout L(*p);
    out->knn_idx = L.at<int32_t>(ws, L.knn_idx);
    out->knn_d2 = L.at<float>(ws, L.knn_d2);
    out->eps = L.at<float>(ws, L.eps);
    out->row_start = L.at<int32_t>(ws, L.row_start);
    out->row_len = L.at<int32_t>(ws, L.row_len);
    out->col = L.at<int32_t>(ws, L.col);
    out->w = L.at<float>(ws, L.w);
    out->d2 = L.at<float>(ws, L.d2e);
    out->deg = L.at<float>(ws, L.deg);
    out->U32 = L.at<float>(ws, L.P) + size_t(L.base) * L.C;
    out->wadj = L.at<float>(ws, L.Wadj) + size_t(L.base) * L.C;
    out->status = L.at<int32_t>(ws, L.status);
    return GLL_OK;
}

int gll_cg_csr(int m, int C, const int32_t* row_ptr, const int32_t* col, const float* val,
               const float* b, float* x, float atol, int max_iter, int32_t* iters,
               int32_t* nonconv, void* workspace, void* stream) {
    if (m < 1 || C < 1 || !row_ptr || !col || !val || !b || !x) return GLL_ERR_INVALID_ARG;
    if (m > 2048 && C <= 16) {   // whole-GPU CG (nnz unknown here: the whole LDS slice)
        if (!workspace) return GLL_ERR_INVALID_ARG;
        prof_begin(GLL_K_CG, static_cast<hipStream_t>(stream));
        const hipError_t e = launch_cg_grid_csr(m, C, row_ptr, col, val, -1, b, x,
                                                atol, max_iter > 0 ? max_iter : 100000, iters,
                                                nonconv, nullptr,
                                                static_cast<float*>(workspace),
                                                static_cast<hipStream_t>(stream));
        prof_end(GLL_K_CG, static_cast<hipStream_t>(stream));
        if (e != hipErrorNotSupported) return hip_status(e);
        // past the grid kernel's capacity: per-column CG with the vectors in the workspace
    }
    return hip_status(launch_cg_csr(m, C, row_ptr, col, val, b, x, atol,
                                    max_iter > 0 ? max_iter : 100000, iters, nonconv,
                                    static_cast<float*>(workspace),
                                    static_cast<hipStream_t>(stream)));
}

size_t gll_cg_csr_workspace_bytes(int m, int C) {
    const size_t per_col = size_t(5) * m * C, grid = grid_cg_workspace_floats(m, C);
    return (per_col > grid ? per_col : grid) * sizeof(float);
}

int gll_set_knob(int id, int value) {
    if (id < 0 || id >= GLL_KNOB_COUNT || value < 0) return GLL_ERR_INVALID_ARG;
    g_knobs[id].store(value, std::memory_order_relaxed);
    return GLL_OK;
}

int gll_prof_enable(int kid, int period) {
    if (kid < 0 || kid >= GLL_K_COUNT || period < 0) return GLL_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(g_prof.mu);
    g_prof.on[kid] = period > 0;
    g_prof.period[kid] = period > 0 ? period : 1;
    g_prof.count[kid] = 0;
    if (g_armed.kid == kid) g_armed = ArmedLaunch{};
    return GLL_OK;
}

int gll_prof_read(int kid, double* ms_total, int* count) {
    if (kid < 0 || kid >= GLL_K_COUNT || !ms_total || !count) return GLL_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(g_prof.mu);
    auto& v = g_prof.pending[kid];
    double tot = 0.0;
    int cnt = 0;
    for (size_t q = 0; q + 1 < v.size(); q += 2) {
        if (hipEventSynchronize(v[q + 1]) != hipSuccess) return GLL_ERR_HIP;
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, v[q], v[q + 1]) != hipSuccess) return GLL_ERR_HIP;
        tot += ms;
        ++cnt;
    }
    for (auto e : v) g_prof.pool.push_back(e);
    v.clear();
    *ms_total = tot;
    *count = cnt;
    return GLL_OK;
}

const char* gll_kernel_name(int kid) {
    if (kid < 0 || kid >= GLL_K_COUNT) return "?";
    return kKernelNames[kid];
}

#ifndef GLL_BUILD_ID
#define GLL_BUILD_ID "unknown"
#endif
const char* gll_build_id(void) { return GLL_BUILD_ID; }

const char* gll_strerror(int code) {
    switch (code) {
        case GLL_OK: return "ok";
        case GLL_ERR_INVALID_ARG: return "invalid argument";
        case GLL_ERR_UNSUPPORTED: return "unsupported problem size (see include/gll.h limits)";
        case GLL_ERR_HIP: return "HIP launch error";
        default: return "unknown error";
    }
}

}  // extern "C"

#ifdef GLL_TRACE
// Diagnostic build only (libgll_trace.so): in-kernel timestamps per translation unit
// (0 knn, 1 rows, 2 solve, 3 grad), see GLL_TRACE_UNIT in gll_internal.h.
namespace gll {
void trace_read_knn(unsigned long long*);
void trace_read_rows(unsigned long long*);
void trace_read_solve(unsigned long long*);
void trace_read_grad(unsigned long long*);
void trace_read_gridcg(unsigned long long*);
void trace_reset_gridcg();
void trace_read_wg_knn(unsigned long long*);
void trace_read_wg_solve(unsigned long long*);
void trace_read_wg_gridcg(unsigned long long*);
void trace_reset_knn();
void trace_reset_rows();
void trace_reset_solve();
void trace_reset_grad();
}  // namespace gll

extern "C" int gll_trace_read(int unit, unsigned long long* out) {
    (void)hipDeviceSynchronize();
    switch (unit) {
        case 0: gll::trace_read_knn(out); return GLL_OK;
        case 1: gll::trace_read_rows(out); return GLL_OK;
        case 2: gll::trace_read_solve(out); return GLL_OK;
        case 3: gll::trace_read_grad(out); return GLL_OK;
        case 4: gll::trace_read_gridcg(out); return GLL_OK;
        default: return GLL_ERR_INVALID_ARG;
    }
}

extern "C" int gll_trace_read_wg(int unit, unsigned long long* out) {
    (void)hipDeviceSynchronize();
    switch (unit) {
        case 0: gll::trace_read_wg_knn(out); return GLL_OK;
        case 2: gll::trace_read_wg_solve(out); return GLL_OK;
        case 4: gll::trace_read_wg_gridcg(out); return GLL_OK;
        default: return GLL_ERR_INVALID_ARG;
    }
}

namespace gll { void trace_read_fz(unsigned long long*); }
extern "C" int gll_trace_read_fz(unsigned long long* out) {
    (void)hipDeviceSynchronize();
    gll::trace_read_fz(out);
    return GLL_OK;
}

extern "C" int gll_trace_reset(int unit) {
    (void)hipDeviceSynchronize();
    switch (unit) {
        case 0: gll::trace_reset_knn(); return GLL_OK;
        case 1: gll::trace_reset_rows(); return GLL_OK;
        case 2: gll::trace_reset_solve(); return GLL_OK;
        case 3: gll::trace_reset_grad(); return GLL_OK;
        case 4: gll::trace_reset_gridcg(); return GLL_OK;
        default: return GLL_ERR_INVALID_ARG;
    }
}
#endif
