// grad.hip -- feature gradient of the Laplace-learning layer.
//
// Replaces the backward tail of /root/reference/GLL.py: the per-class loop over
// graph.gradient (GLL.py:111-120), the self-tuning-eps term (GLL.py:124-139) and the
// Laplacian SpMM laplacian(G o V) @ X (GLL.py:146-159), in closed form:
//     G_ij = sum_c (w_ic - w_jc)(P_jc - P_ic),  V_ij = -8 W_ij / (eps_i eps_j),  S = G V
//     grad_i = sum_j coef_ij (x_i - x_j)
//     coef_ij = S_ij                                                  (fixed eps)
//     coef_ij = S_ij - b_i [j = kth(i)] - b_j [kth(j) = i]            (auto eps)
//     b_i = sum_j G_ij d_ij^2 V_ij / (2 eps_i^2)
// Both kinds of extra term sit on graph edges (kth(i) is a neighbour of i), so the whole
// backward is ONE pass over the CSR (fixed eps) or two (auto eps: b must be complete
// before any row uses its neighbours' b).  One wave per row; lanes first own edges
// (coefficients), then own feature columns (the x_j gathers, 16-B coalesced per lane).
#include "gll_internal.h"
#include "grad_common.h"

namespace gll {

GLL_TRACE_UNIT(grad)

// auto eps, pass 1: S_ij and b_i (also the fixed-eps S_ij of the feature-chunked gradient).
// LPR lanes per row (rows are ~K..2K edges: a whole wave per row left most lanes idle), CV the
// class bound of the register form (0: the generic loop).  Latency-bound -- three dependent
// gathers per edge -- so the register budget (occupancy) is what the CV templating buys.
template <int CV, int LPR>
__global__ __launch_bounds__(256) void edge_coef_kernel(EdgeArgs a) {
    GLL_TRACE_SCOPE(0);
    a.to_graph();
    constexpr int RPW = kWave / LPR;
    const int lane = lane_id();
    const int gl = lane % LPR;
    const int i = bx() * (4 * RPW) + (threadIdx.x >> 6) * RPW + lane / LPR;
    const bool live = i < a.n;
    const int ic = live ? i : 0;
    const int beg = live ? a.row_start[ic] : 0;
    const int end = live ? beg + a.row_len[ic] : 0;
    const float ei = a.eps_fixed > 0.f ? a.eps_fixed : a.eps[ic];
    float bpart = 0.f;
    if constexpr (CV != 0) {
        const auto ri = row_wp<CV>(a, ic);
        for (int e = beg + gl; e < end; e += LPR) {
            const float s = edge_gv_r<CV>(a, ri, a.col[e], a.w[e], ei);
            a.S[e] = s;
            bpart += s * a.d2[e];   // G d^2 V
        }
    } else {
        for (int e = beg + gl; e < end; e += LPR) {
            float g;
            const float s = edge_gv(a, ic, a.col[e], a.w[e], ei, g);
            a.S[e] = s;
            bpart += s * a.d2[e];   // G d^2 V
        }
    }
#pragma unroll
    for (int o = LPR / 2; o > 0; o >>= 1) bpart += __shfl_xor(bpart, o, LPR);
    if (live && gl == 0) a.b[i] = bpart / (2.f * ei * ei);  // modV = d^2 V / (2 eps_i^2), GLL.py:218
}

template <int CV>
static void launch_edge_coef(const EdgeArgs& a, const Batch& bt, int lpr, hipStream_t s) {
    const unsigned rows = 4u * unsigned(kWave / lpr);
    const dim3 grid((unsigned(a.n) + rows - 1) / rows, bt.B);
    if (lpr == 16) launch_k(edge_coef_kernel<CV, 16>, grid, 256, 0, s, a);
    else if (lpr == 32) launch_k(edge_coef_kernel<CV, 32>, grid, 256, 0, s, a);
    else launch_k(edge_coef_kernel<CV, 64>, grid, 256, 0, s, a);
}

// out_i = sum_e coef_e (x_i - x_{col_e}) in the difference form: translation-invariant like the
// closed form (the reference's laplacian(S) @ X, GLL.py:146-159, cancels (sum coef) x_i against
// sum coef x_j in fp32 and loses |x| / |x_i - x_j| of its digits on offset features; the fp32
// differences of nearby rows are exact).  AUTO selects the coefficient form
// WIDE (single-graph launches, where occupancy is not the limit): twice the x_j rows in
// flight per batch -- an NS row's ~13 neighbours in one memory round trip instead of two.
// CV (fixed eps): the class bound of the inline coefficient, as in edge_coef_kernel -- row i's
// w and P in registers and all 2C loads of row j in one round trip (-C exact even count, > 0 a
// bound, 0 the generic loop: C dependent round trips per edge, which dominated the batched NS
// gradient).  Same fma order, so every form agrees bitwise.
template <bool AUTO, int ND, bool VEC, bool WIDE, int CV>
__global__ __launch_bounds__(256) void grad_spmm_kernel(EdgeArgs a, const float* __restrict__ X,
                                                        float* __restrict__ out, size_t xs,
                                                        size_t gxs) {
    GLL_TRACE_SCOPE(1);
    const int2 xy = batch_xy<true>();   // once: (block within the graph, graph)
    a.to_graph_at(xy.y);
    X = gshift_at(X, xs, xy.y);
    out = gshift_at(out, gxs, xy.y);
    const int lane = lane_id();
    const int i = xy.x * 4 + (threadIdx.x >> 6);
    if (i >= a.n) return;
    const int d = a.d;
    const int beg = a.row_start[i], end = beg + a.row_len[i];
    const float ei = a.eps_fixed > 0.f ? a.eps_fixed : a.eps[i];
    const float* xi = X + size_t(i) * d;
    // x_i, loaded up front: its latency hides behind the edge loop.  Rows are read unmasked
    // (load4_raw: lanes past d read in-bounds clamped addresses, and their sums are never stored)
    f32x4 xv[ND];
#pragma unroll
    for (int q = 0; q < ND; ++q) xv[q] = load4_raw<VEC>(xi, 4 * lane + 4 * kWave * q, d);
    int kth_i = 0;
    float b_i = 0.f;
    if constexpr (AUTO) {
        kth_i = a.knn_idx[size_t(i) * a.K + a.K - 1];
        b_i = a.b[i];
    }
    f32x4 acc[ND];
#pragma unroll
    for (int q = 0; q < ND; ++q) acc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int e0 = beg; e0 < end; e0 += kWave) {
        // lanes own edges: coefficient of edge e0 + lane
        const int e = e0 + lane;
        float cf = 0.f;
        int cj = i;
        // row i's w and P for the register form (fixed eps), loaded per 64 edges so they are
        // dead during the gathers below (VGPRs = occupancy); AUTO or CV = 0: unused
        const auto ri = row_wp<(AUTO || CV == 0) ? 1 : CV>(a, (AUTO || CV == 0) ? 0 : i);
        if (e < end) {
            cj = a.col[e];
            if constexpr (AUTO) {
                cf = a.S[e];
                if (cj == kth_i) cf -= b_i;
                if (a.knn_idx[size_t(cj) * a.K + a.K - 1] == i) cf -= a.b[cj];
            } else if constexpr (CV != 0) {
                cf = edge_gv_r<CV>(a, ri, cj, a.w[e], ei);
            } else {
                float g;
                cf = edge_gv(a, i, cj, a.w[e], ei, g);
            }
        }
        // lanes own feature columns: accumulate coef_e * x_j in edge order, EB rows of X in
        // flight per batch (padded slots carry coefficient 0 on row i itself)
        const int cnt = min(kWave, end - e0);
        // batches (not WIDE) at ND = 2 take 4 rows per batch: 70 instead of 110 VGPRs, 7 waves
        // per SIMD instead of 4 (B = 64 NS 182 -> 170 us)
        constexpr int EB0 = ND <= 2 ? 8 : (ND <= 4 ? 4 : (ND <= 8 ? 2 : 1));
        constexpr int EB = WIDE ? 2 * EB0 : (ND == 2 ? 4 : EB0);
        for (int t0 = 0; t0 < cnt; t0 += EB) {
            float s[EB];
            f32x4 v[EB][ND];
#pragma unroll
            for (int u = 0; u < EB; ++u) {
                const int t = t0 + u < cnt ? t0 + u : t0;
                s[u] = t0 + u < cnt ? readlane_f(cf, t) : 0.f;
                const float* xj = X + size_t(readlane_i(cj, t)) * d;
#pragma unroll
                for (int q = 0; q < ND; ++q) v[u][q] = load4_raw<VEC>(xj, 4 * lane + 4 * kWave * q, d);
            }
#pragma unroll
            for (int u = 0; u < EB; ++u) {
#pragma unroll
                for (int q = 0; q < ND; ++q) acc[q] += s[u] * (xv[q] - v[u][q]);
            }
        }
    }
    float* oi = out + size_t(i) * d;
#pragma unroll
    for (int q = 0; q < ND; ++q) {
        const int k = 4 * lane + 4 * kWave * q;
        const f32x4 r = acc[q];
        if constexpr (VEC) {
            if (k < d) __builtin_nontemporal_store(r, reinterpret_cast<f32x4*>(oi + k));   // streamed out: not re-read here
        } else {
            if (k + 0 < d) oi[k + 0] = r.x;
            if (k + 1 < d) oi[k + 1] = r.y;
            if (k + 2 < d) oi[k + 2] = r.z;
            if (k + 3 < d) oi[k + 3] = r.w;
        }
    }
}

// Feature-chunked form: the same sums with the features split into NCH chunks of 4 LPR floats,
// block b taking chunk b % NCH.  Blocks are dealt round-robin over the 8 XCDs, so with NCH | 8
// each XCD gathers only its own chunk of the neighbour rows: its working set is n x d / NCH x 4 B
// (4 MB at stress, d = 1024, NCH = 8), which its L2 holds, instead of all of X (32 MB) streamed
// from the MALL once per edge.  LPR lanes own one row (RPW = 64 / LPR rows per wave): they first
// own the row's edges (coefficients), then its chunk's feature columns; an edge's coefficient and
// column reach the group's lanes by a width-LPR shuffle.  The per-edge coefficient is recomputed
// per chunk (C-wide gathers from the n x C arrays, L2-resident).  Same edge order and summation
// per element as grad_spmm_kernel, so the two agree bitwise.
// COEF: 1 = auto eps (S and b from edge_coef_kernel); 2 = fixed eps, S from edge_coef_kernel
// (an inline G V would be recomputed by every chunk: 2C + 1 gathers per edge, which at NCH = 8
// cost more than the chunking saves).
template <int COEF, int LPR>
__global__ __launch_bounds__(256) void grad_chunk_kernel(EdgeArgs a, const float* __restrict__ X,
                                                         float* __restrict__ out, int nch,
                                                         size_t xs, size_t gxs,
                                                         const int32_t* __restrict__ perm,
                                                         const int32_t* __restrict__ perm_ok) {
    GLL_TRACE_SCOPE(1);
    a.to_graph();
    // the order exists only if this workspace's forward wrote it (its flags may differ from the
    // backward's: gll_backward takes its own gll_problem)
    if (perm && *perm_ok != 1) perm = nullptr;
    X = gshift(X, xs);
    out = gshift(out, gxs);
    constexpr int RPW = kWave / LPR;
    constexpr int EB = LPR >= 32 ? 8 : 16;   // neighbour rows in flight per lane
    const int lane = lane_id();
    const int gl = lane % LPR;                // lane inside the row's group
    const int blk = bx();
    const int chunk = blk % nch;
    // row position in time order: the locality order of a large graph (gll_internal.h
    // locality_order) when given, so a chunk's XCD gathers the neighbour rows of nearby rows
    const int pos = (blk / nch) * (4 * RPW) + (threadIdx.x >> 6) * RPW + lane / LPR;
    const bool live = pos < a.n;
    const int i = live ? (perm ? perm[pos] : pos) : pos;
    const int ic = live ? i : 0;
    const int d = a.d;
    const int k = chunk * 4 * LPR + 4 * gl;   // this lane's 4 features
    const bool kin = k < d;
    const int kc = kin ? k : 0;
    const int beg = live ? a.row_start[ic] : 0;
    const int end = live ? beg + a.row_len[ic] : 0;
    const float ei = a.eps_fixed > 0.f ? a.eps_fixed : a.eps[ic];
    const f32x4 xv = *reinterpret_cast<const f32x4*>(X + size_t(ic) * d + kc);
    int kth_i = 0;
    float b_i = 0.f;
    if constexpr (COEF == 1) {
        kth_i = a.knn_idx[size_t(ic) * a.K + a.K - 1];
        b_i = a.b[ic];
    }
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int e0 = beg; e0 < end; e0 += LPR) {
        const int e = e0 + gl;
        float cf = 0.f;
        int cj = ic;
        if (e < end) {
            cj = a.col[e];
            if constexpr (COEF == 1) {
                cf = a.S[e];
                if (cj == kth_i) cf -= b_i;
                if (a.knn_idx[size_t(cj) * a.K + a.K - 1] == i) cf -= a.b[cj];
            } else {
                cf = a.S[e];
            }
        }
        const int cnt = min(LPR, end - e0);
        for (int t0 = 0; t0 < cnt; t0 += EB) {
            float s[EB];
            f32x4 v[EB];
#pragma unroll
            for (int u = 0; u < EB; ++u) {
                const int t = t0 + u < cnt ? t0 + u : t0;
                s[u] = __shfl(cf, t, LPR);
                s[u] = t0 + u < cnt ? s[u] : 0.f;
                const int j = __shfl(cj, t, LPR);
                v[u] = *reinterpret_cast<const f32x4*>(X + size_t(j) * d + kc);
            }
#pragma unroll
            for (int u = 0; u < EB; ++u) acc += s[u] * (xv - v[u]);
        }
    }
    if (live && kin)
        __builtin_nontemporal_store(acc, reinterpret_cast<f32x4*>(out + size_t(i) * d + k));
}

// Whether the feature-chunked gradient runs: 16-B rows with d >= 128, and either a graph whose X
// does not fit an XCD's 4 MB L2 or a batch of narrow graphs (d < 256, where a wave per row
// leaves lanes idle), or forced by the flags.  Measured (tools/ab_flags.py --flags 0,2048,
// edge coefficients + gradient): stress 16 + 94 vs 194 us; FullySup B = 64 61 + 102 vs 309 us;
// NS B = 64 26 + 146 vs 170 us and NS/FullySup single graphs a tie (X already fits; the
// chunks only add the coefficient pass).
static bool grad_use_chunks(const Layout& L, const Batch& bt, bool vec) {
    if (!vec || L.d < 128 || (L.d & 3) || (L.flags & GLL_FLAG_GRAD_ROWS)) return false;
    return (L.flags & GLL_FLAG_GRAD_CHUNK) || (bt.B > 1 && L.d < 256) ||
           size_t(L.n) * L.d * 4 > (size_t(4) << 20);
}

// LPR = the power of two nearest d / 32 in [16, 64], NCH = ceil(d / (4 LPR)) chunks.
template <int COEF>
static void grad_chunked(const EdgeArgs& a, const Batch& bt, const float* X, float* out,
                         const int32_t* perm, const int32_t* perm_ok, hipStream_t s) {
    int lpr = 16;
    while (lpr < 64 && 4 * lpr * 8 < a.d) lpr *= 2;
    const int nch = (a.d + 4 * lpr - 1) / (4 * lpr);
    const int rows_per_block = 4 * (kWave / lpr);
    dim3 grid(unsigned(nch * ((a.n + rows_per_block - 1) / rows_per_block)), bt.B);
    if (lpr == 16)
        launch_k(grad_chunk_kernel<COEF, 16>, grid, 256, 0, s, a, X, out, nch, bt.x, bt.gx, perm,
                 perm_ok);
    else if (lpr == 32)
        launch_k(grad_chunk_kernel<COEF, 32>, grid, 256, 0, s, a, X, out, nch, bt.x, bt.gx, perm,
                 perm_ok);
    else
        launch_k(grad_chunk_kernel<COEF, 64>, grid, 256, 0, s, a, X, out, nch, bt.x, bt.gx, perm,
                 perm_ok);
}

template <bool AUTO, bool VEC, int CV>
static hipError_t grad_nd(const EdgeArgs& a, const Batch& bt, const float* X, float* out,
                          hipStream_t s) {
    dim3 grid((a.n + 3) / 4, bt.B);
    const int nd = (a.d + 255) / 256;
#define GLL_GRAD(ND)                                                                        \
    do {                                                                                    \
        if (bt.B == 1 && ND <= 4)                                                           \
            launch_k(grad_spmm_kernel<AUTO, ND, VEC, true, CV>, grid, 256, 0, s, a, X, out, bt.x, bt.gx);  \
        else                                                                                \
            launch_k(grad_spmm_kernel<AUTO, ND, VEC, false, CV>, grid, 256, 0, s, a, X, out, bt.x, bt.gx); \
    } while (0)
    if (nd <= 1) GLL_GRAD(1);
    else if (nd <= 2) GLL_GRAD(2);
    else if (nd <= 4) GLL_GRAD(4);
    else if (nd <= 8) GLL_GRAD(8);
    else if (nd <= 16) GLL_GRAD(16);
    else return hipErrorInvalidValue;
#undef GLL_GRAD
    return launch_status("grad.hip:grad_nd");
}

hipError_t launch_backward_grad(const Layout& L, const Batch& bt, void* ws, const float* X,
                                bool auto_eps, float eps_fixed, float* gradX, bool vec,
                                hipStream_t s) {
    const EdgeArgs a = make_edge_args(L, bt.ws, ws, auto_eps ? 0.f : eps_fixed);
    hipError_t e;
    const bool chunk = grad_use_chunks(L, bt, vec);
    if (auto_eps || chunk) {   // per-edge S (and b) first
        const int lpr = L.K <= 40 ? 16 : 32;   // tools/ab_flags.py: 16 lanes per row beat 32/64
        prof_begin(GLL_K_EDGE, s);
        switch (L.C) {   // even C <= 16: exact count, paired loads; else a bound, or the loop
            case 2: launch_edge_coef<-2>(a, bt, lpr, s); break;
            case 4: launch_edge_coef<-4>(a, bt, lpr, s); break;
            case 6: launch_edge_coef<-6>(a, bt, lpr, s); break;
            case 8: launch_edge_coef<-8>(a, bt, lpr, s); break;
            case 10: launch_edge_coef<-10>(a, bt, lpr, s); break;
            case 12: launch_edge_coef<-12>(a, bt, lpr, s); break;
            case 14: launch_edge_coef<-14>(a, bt, lpr, s); break;
            case 16: launch_edge_coef<-16>(a, bt, lpr, s); break;
            default:
                if (L.C <= 4) launch_edge_coef<4>(a, bt, lpr, s);
                else if (L.C <= 8) launch_edge_coef<8>(a, bt, lpr, s);
                else if (L.C <= 16) launch_edge_coef<16>(a, bt, lpr, s);
                else launch_edge_coef<0>(a, bt, lpr, s);
        }
        prof_end(GLL_K_EDGE, s);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    prof_begin(GLL_K_GRAD, s);
    if (chunk) {
        // the forward's order, if it wrote one (device word: the forward's flags are not known here)
        const bool order = bt.B == 1 && L.PR == L.n && L.n >= 16 * kPiv &&
                           size_t(L.n) * L.d * 4 > (size_t(4) << 20);
        const int32_t* perm = order ? L.at<int32_t>(ws, L.perm) : nullptr;
        const int32_t* pok = L.at<int32_t>(ws, L.status) + kStPermValid;
        if (auto_eps) grad_chunked<1>(a, bt, X, gradX, perm, pok, s);
        else grad_chunked<2>(a, bt, X, gradX, perm, pok, s);
        e = launch_status("grad.hip:grad_chunked");
    } else if (auto_eps) {
        e = vec ? grad_nd<true, true, 0>(a, bt, X, gradX, s)
                : grad_nd<true, false, 0>(a, bt, X, gradX, s);
    } else {
        // fixed eps: inline coefficient in register form for ten classes (every caller's label
        // matrix, FullySup.py:153; other C the generic loop)
        if (L.C == 10)
            e = vec ? grad_nd<false, true, -10>(a, bt, X, gradX, s)
                    : grad_nd<false, false, -10>(a, bt, X, gradX, s);
        else
            e = vec ? grad_nd<false, true, 0>(a, bt, X, gradX, s)
                    : grad_nd<false, false, 0>(a, bt, X, gradX, s);
    }
    prof_end(GLL_K_GRAD, s);
    return e;
}

}  // namespace gll
