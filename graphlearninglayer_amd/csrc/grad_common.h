// grad_common.h -- per-edge pieces of the feature gradient shared by grad.hip and the fused
// adjoint-CG + gradient kernel of solve.hip (closed form of GLL.py:111-159):
//     G_ij = sum_c (w_ic - w_jc)(P_jc - P_ic),  V_ij = -8 W_ij / (eps_i eps_j)
#pragma once

#include "gll_internal.h"

namespace gll {

struct EdgeArgs {
    int n, base, C, K, d;
    float eps_fixed;      // > 0: every eps_i equals it (fixed epsilon) -- no eps gathers
    const int32_t* row_start;
    const int32_t* row_len;
    const int32_t* col;
    const float* w;       // W_ij
    const float* d2;      // d_ij^2
    const float* eps;
    const float* P;       // n x C  [Y; U]
    const float* Wadj;    // n x C  [0; Luu^-1 gbar]
    const int32_t* knn_idx;
    float* S;             // per-edge S (auto)
    float* b;             // per-row b (auto)
    size_t wss;           // batched launches: workspace stride between graphs (bytes)

    template <bool R = false>
    __device__ void to_graph() { to_graph_at(bg<R>()); }
    __device__ void to_graph_at(int g) {   // move every workspace pointer to graph g
        row_start = gshift_at(row_start, wss, g);
        row_len = gshift_at(row_len, wss, g);
        col = gshift_at(col, wss, g);
        w = gshift_at(w, wss, g);
        d2 = gshift_at(d2, wss, g);
        eps = gshift_at(eps, wss, g);
        P = gshift_at(P, wss, g);
        Wadj = gshift_at(Wadj, wss, g);
        knn_idx = gshift_at(knn_idx, wss, g);
        S = gshift_at(S, wss, g);
        b = gshift_at(b, wss, g);
    }
};

// G_ij * V_ij for edge e = (i, j)
__device__ __forceinline__ float edge_gv(const EdgeArgs& a, int i, int j, float we, float ei,
                                         float& gout) {
    const float* wi = a.Wadj + size_t(i) * a.C;
    const float* wj = a.Wadj + size_t(j) * a.C;
    const float* pi = a.P + size_t(i) * a.C;
    const float* pj = a.P + size_t(j) * a.C;
    float g = 0.f;
    for (int c = 0; c < a.C; ++c) g = __builtin_fmaf(wi[c] - wj[c], pj[c] - pi[c], g);
    gout = g;
    const float ej = a.eps_fixed > 0.f ? a.eps_fixed : a.eps[j];
    const float v = -8.f * we / (ei * ej);   // GLL.py:217/234
    return g * v;
}

// The same with row i's values of w and P already in registers and the class count a
// compile-time bound CV >= C: all 2C loads of row j are issued before any is used (the loop
// above is one dependent L2 round trip per class), and the sum runs in the same order with
// explicit fmas (the unrolled form is otherwise vectorised into packed multiplies and adds,
// which round twice), so the two agree bitwise.
template <int CV>
struct RowWP {
    float w[CV], p[CV];
};
// CV < 0: exactly -CV classes (even), rows loaded as 8-B pairs (the n x C rows are 8-B aligned
// when C is even) -- C / 2 loads per array instead of CV.
template <int CV>
__device__ __forceinline__ void load_wp(const EdgeArgs& a, int i, float* w, float* p) {
    constexpr int N = CV < 0 ? -CV : CV;
    const float* wi = a.Wadj + size_t(i) * a.C;
    const float* pi = a.P + size_t(i) * a.C;
    if constexpr (CV < 0) {
        typedef float f32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int c = 0; c < N; c += 2) {
            const f32x2 u = *reinterpret_cast<const f32x2*>(wi + c);
            const f32x2 v = *reinterpret_cast<const f32x2*>(pi + c);
            w[c] = u.x, w[c + 1] = u.y, p[c] = v.x, p[c + 1] = v.y;
        }
    } else {
#pragma unroll
        for (int c = 0; c < N; ++c) {
            const int cc = c < a.C ? c : 0;
            w[c] = wi[cc];
            p[c] = pi[cc];
        }
    }
}
template <int CV>
__device__ __forceinline__ RowWP<CV < 0 ? -CV : CV> row_wp(const EdgeArgs& a, int i) {
    RowWP<CV < 0 ? -CV : CV> r;
    load_wp<CV>(a, i, r.w, r.p);
    return r;
}
template <int CV>
__device__ __forceinline__ float edge_gv_r(const EdgeArgs& a, const RowWP<CV < 0 ? -CV : CV>& ri,
                                           int j, float we, float ei) {
    constexpr int N = CV < 0 ? -CV : CV;
    float wv[N], pv[N];
    load_wp<CV>(a, j, wv, pv);
    float g = 0.f;
#pragma unroll
    for (int c = 0; c < N; ++c)
        if (CV < 0 || c < a.C) g = __builtin_fmaf(ri.w[c] - wv[c], pv[c] - ri.p[c], g);
    const float ej = a.eps_fixed > 0.f ? a.eps_fixed : a.eps[j];
    const float v = -8.f * we / (ei * ej);   // GLL.py:217/234
    return g * v;
}

// The workspace arrays of graph 0 (eps_fixed <= 0: auto eps, eps gathered per row).
inline EdgeArgs make_edge_args(const Layout& L, size_t wss, void* ws, float eps_fixed) {
    EdgeArgs a;
    a.n = L.n;
    a.base = L.base;
    a.C = L.C;
    a.K = L.K;
    a.d = L.d;
    a.eps_fixed = eps_fixed > 0.f ? eps_fixed : 0.f;
    a.row_start = L.at<int32_t>(ws, L.row_start);
    a.row_len = L.at<int32_t>(ws, L.row_len);
    a.col = L.at<int32_t>(ws, L.col);
    a.w = L.at<float>(ws, L.w);
    a.d2 = L.at<float>(ws, L.d2e);
    a.eps = L.at<float>(ws, L.eps);
    a.P = L.at<float>(ws, L.P);
    a.Wadj = L.at<float>(ws, L.Wadj);
    a.knn_idx = L.at<int32_t>(ws, L.knn_idx);
    a.S = L.at<float>(ws, L.S);
    a.b = L.at<float>(ws, L.b);
    a.wss = wss;
    return a;
}

}  // namespace gll
