// knn.hip -- exact brute-force kNN for the GLL graph (replaces the annoy search of
// graphlearning.weightmatrix.knnsearch, /root/reference/GLL.py:183).
//
//  K1a gram_d2_kernel   D2 = |x_i|^2 + |x_j|^2 - 2 X X^T  on fp32 MFMA (v_mfma_f32_32x32x2_f32)
//                       64x64 output tile per 256-thread workgroup, one 32x32 tile per wave,
//                       operands streamed straight to VGPRs (the f32 MFMA needs one VGPR per
//                       operand per lane), row norms accumulated from the same loads.
//  K1b knn_select_kernel one wave per row: per-lane sorted candidate lists over the D2 row,
//                       a 64-lane merge to kc = K-1+margin candidates, exact re-ranking with
//                       d^2 = sum_k (x_ik - x_jk)^2 (bitwise symmetric in i,j), then the K-1
//                       nearest with ties broken by index.  Self is forced to rank 0 with
//                       distance 0 (the stand-in contract of SURVEY.md §8c).
#include <limits.h>

#include "gll_internal.h"

namespace gll {

// --------------------------------------------------------------------------------------
// K1a: Gram / squared-distance tile
// --------------------------------------------------------------------------------------
template <bool VEC>
__global__ __launch_bounds__(256) void gram_d2_kernel(const float* __restrict__ X, int n, int d,
                                                      float* __restrict__ D2, int ld,
                                                      int32_t* __restrict__ status) {
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    const int r = lane & 31;   // A row / B column owned by this lane
    const int h = lane >> 5;   // k half: lane holds k = k0 + 4h + t, t = 0..3
    const int row0 = blockIdx.y * 64 + (wave >> 1) * 32;
    const int col0 = blockIdx.x * 64 + (wave & 1) * 32;
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x < GLL_ST_NWORDS) status[threadIdx.x] = 0;

    const float* pa = X + size_t(min(row0 + r, n - 1)) * d + 4 * h;
    const float* pb = X + size_t(min(col0 + r, n - 1)) * d + 4 * h;
    const int lim = d - 4 * h;

    f32x16 acc;
#pragma unroll
    for (int g = 0; g < 16; ++g) acc[g] = 0.f;
    float sa = 0.f, sb = 0.f;

    constexpr int U = 4;  // 4 steps x 8 k = 32 k per chunk, one chunk prefetched ahead
    f32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        a[u] = load4<VEC>(pa, 8 * u, lim);
        b[u] = load4<VEC>(pb, 8 * u, lim);
    }
    for (int k0 = 0; k0 < d; k0 += 8 * U) {
        f32x4 an[U], bn[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            an[u] = load4<VEC>(pa, k0 + 8 * U + 8 * u, lim);
            bn[u] = load4<VEC>(pb, k0 + 8 * U + 8 * u, lim);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            sa += a[u].x * a[u].x + a[u].y * a[u].y + a[u].z * a[u].z + a[u].w * a[u].w;
            sb += b[u].x * b[u].x + b[u].y * b[u].y + b[u].z * b[u].z + b[u].w * b[u].w;
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].x, b[u].x, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].y, b[u].y, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].z, b[u].z, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u].w, b[u].w, acc, 0, 0, 0);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            a[u] = an[u];
            b[u] = bn[u];
        }
    }
    // full row norms: lanes r and r+32 hold the two k halves of row r
    sa += __shfl_xor(sa, 32);
    sb += __shfl_xor(sb, 32);
    const int j = col0 + r;
    // C/D layout of the 32x32 MFMA: col = lane & 31, row = (g & 3) + 8 (g >> 2) + 4 (lane >> 5)
#pragma unroll
    for (int g = 0; g < 16; ++g) {
        const int ii = (g & 3) + 8 * (g >> 2) + 4 * h;
        const float sqi = __shfl(sa, ii);
        const int i = row0 + ii;
        if (i < n && j < n) D2[size_t(i) * ld + j] = sqi + sb - 2.f * acc[g];
    }
}

// --------------------------------------------------------------------------------------
// K1b: per-row selection + exact re-rank
// --------------------------------------------------------------------------------------
template <int KC>
__device__ __forceinline__ void list_insert(float (&key)[KC], int (&idx)[KC], float v, int j) {
    // precondition: v < key[KC-1]; keeps ascending order, equal keys keep scan order
#pragma unroll
    for (int t = KC - 1; t > 0; --t) {
        const bool shift = key[t - 1] > v;
        const bool here = key[t] > v;
        key[t] = shift ? key[t - 1] : (here ? v : key[t]);
        idx[t] = shift ? idx[t - 1] : (here ? j : idx[t]);
    }
    const bool here0 = key[0] > v;
    key[0] = here0 ? v : key[0];
    idx[0] = here0 ? j : idx[0];
}

template <int KC>
__device__ __forceinline__ void list_pop(float (&key)[KC], int (&idx)[KC], bool pop) {
#pragma unroll
    for (int t = 0; t < KC - 1; ++t) {
        key[t] = pop ? key[t + 1] : key[t];
        idx[t] = pop ? idx[t + 1] : idx[t];
    }
    key[KC - 1] = pop ? __builtin_inff() : key[KC - 1];
    idx[KC - 1] = pop ? INT_MAX : idx[KC - 1];
}

__device__ __forceinline__ bool lex_less(float ka, int ia, float kb, int ib) {
    return ka < kb || (ka == kb && ia < ib);
}

template <int KC, bool VEC>
__global__ __launch_bounds__(256) void knn_select_kernel(
    const float* __restrict__ D2, int ld, const float* __restrict__ X, int n, int d, int K,
    int kc, float eps_fixed, int auto_eps, int32_t* __restrict__ knn_idx,
    float* __restrict__ knn_d2, float* __restrict__ eps, int32_t* __restrict__ fwd_cnt,
    int32_t* __restrict__ rev_cnt, int32_t* __restrict__ fill_cnt, int32_t* __restrict__ status) {
    const int lane = lane_id();
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;  // whole wave

    float key[KC];
    int idx[KC];
#pragma unroll
    for (int t = 0; t < KC; ++t) {
        key[t] = __builtin_inff();
        idx[t] = INT_MAX;
    }
    // 1) per-lane scan of the row (16-B loads: lane covers 4 consecutive columns)
    const float* row = D2 + size_t(i) * ld;
    for (int j0 = 4 * lane; j0 < n; j0 += 4 * kWave) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(row + j0);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int j = j0 + t;
            const float x = v[t];
            if (j < n && j != i && x < key[KC - 1]) list_insert<KC>(key, idx, x, j);
        }
    }
    // 2) merge: round t hands the t-th smallest (key, idx) to lane t
    int ci = INT_MAX;
    for (int t = 0; t < kc; ++t) {
        float bk = key[0];
        int bi = idx[0];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const float ok = __shfl_xor(bk, off);
            const int oi = __shfl_xor(bi, off);
            if (lex_less(ok, oi, bk, bi)) {
                bk = ok;
                bi = oi;
            }
        }
        if (lane == t) ci = bi;
        list_pop<KC>(key, idx, bi != INT_MAX && idx[0] == bi);
    }
    // 3) exact squared distances of the candidates, lanes across the feature dimension
    const float* xi = X + size_t(i) * d;
    float ce = __builtin_inff();
    for (int t = 0; t < kc; ++t) {
        const int j = readlane_i(ci, t);
        if (j == INT_MAX) continue;  // wave-uniform
        const float* xj = X + size_t(j) * d;
        float part = 0.f;
        for (int k = 4 * lane; k < d; k += 4 * kWave) {
            const f32x4 a = load4<VEC>(xi, k, d);
            const f32x4 bb = load4<VEC>(xj, k, d);
            const f32x4 df = a - bb;
            part += df.x * df.x;
            part += df.y * df.y;
            part += df.z * df.z;
            part += df.w * df.w;
        }
        part = wave_sum(part);
        if (lane == t) ce = part;
    }
    // 4) rank the candidates by (exact d^2, index); keep the K-1 nearest
    int rank = 0;
    for (int u = 0; u < kc; ++u) {
        const float eu = __shfl(ce, u);
        const int iu = __shfl(ci, u);
        rank += (iu != INT_MAX && lex_less(eu, iu, ce, ci)) ? 1 : 0;
    }
    const bool keep = lane < kc && ci != INT_MAX && rank < K - 1;
    int32_t* oi = knn_idx + size_t(i) * K;
    float* od = knn_d2 + size_t(i) * K;
    if (lane == 0) {
        oi[0] = i;
        od[0] = 0.f;
    }
    if (keep) {
        oi[1 + rank] = ci;
        od[1 + rank] = ce;
    }
    // rows with fewer valid candidates (non-finite input) fall back to self, distance 0,
    // i.e. dropped edges (sparse.find drops zeros, GLL.py:198)
    const int nkeep = wave_sum_i(keep ? 1 : 0);
    if (lane >= nkeep && lane < K - 1) {
        oi[1 + lane] = i;
        od[1 + lane] = 0.f;
    }
    const int nfwd = wave_sum_i((keep && ce > 0.f) ? 1 : 0);
    float ei = eps_fixed;
    if (auto_eps) {
        // eps_i = d(i, knn_ind[i, K-1])  (GLL.py:205)
        float e = (keep && rank == K - 2) ? sqrtf(ce) : 0.f;
        ei = wave_sum(e);
    }
    if (lane == 0) {
        fwd_cnt[i] = nfwd;
        rev_cnt[i] = 0;
        fill_cnt[i] = 0;
        eps[i] = ei;
        if (!(ei >= 1e-10f)) atomicOr(&status[GLL_ST_TINY_EPS], 1);  // GLL.py:240-241
    }
}

hipError_t launch_gram(const float* X, int n, int d, float* D2, int ldD, int32_t* status,
                       bool vec, hipStream_t s) {
    dim3 grid((n + 63) / 64, (n + 63) / 64);
    prof_begin(GLL_K_GRAM, s);
    if (vec) gram_d2_kernel<true><<<grid, 256, 0, s>>>(X, n, d, D2, ldD, status);
    else gram_d2_kernel<false><<<grid, 256, 0, s>>>(X, n, d, D2, ldD, status);
    prof_end(GLL_K_GRAM, s);
    return hipGetLastError();
}

hipError_t launch_select(const float* D2, int ldD, const float* X, int n, int d, int K,
                         float eps_fixed, bool auto_eps, int32_t* knn_idx, float* knn_d2,
                         float* eps, int32_t* fwd_cnt, int32_t* rev_cnt, int32_t* fill_cnt,
                         int32_t* status, bool vec, hipStream_t s) {
    // candidate list capacity: smallest of {16, 32, 64} leaving a re-rank margin >= 4
    const int need = K - 1 + 4;
    const int KC = need <= 16 ? 16 : (need <= 32 ? 32 : 64);
    if (K - 1 > 64) return hipErrorInvalidValue;
    int margin = KC - (K - 1);
    if (margin > 8) margin = 8;
    int kc = K - 1 + margin;
    if (kc > n - 1) kc = n - 1;
    dim3 grid((n + 3) / 4);
    prof_begin(GLL_K_SELECT, s);
#define GLL_SEL(KCV, V)                                                                        \
    knn_select_kernel<KCV, V><<<grid, 256, 0, s>>>(D2, ldD, X, n, d, K, kc, eps_fixed,         \
                                                   auto_eps ? 1 : 0, knn_idx, knn_d2, eps,     \
                                                   fwd_cnt, rev_cnt, fill_cnt, status)
    if (KC == 16) { if (vec) GLL_SEL(16, true); else GLL_SEL(16, false); }
    else if (KC == 32) { if (vec) GLL_SEL(32, true); else GLL_SEL(32, false); }
    else { if (vec) GLL_SEL(64, true); else GLL_SEL(64, false); }
#undef GLL_SEL
    prof_end(GLL_K_SELECT, s);
    return hipGetLastError();
}

}  // namespace gll
