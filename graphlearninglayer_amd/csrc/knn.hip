// knn.hip -- exact brute-force kNN for the GLL graph (replaces the annoy search of
// graphlearning.weightmatrix.knnsearch, /root/reference/GLL.py:183).
//
//  K1a gram_d2_kernel   D2 = |x_i|^2 + |x_j|^2 - 2 X X^T  on fp32 MFMA (v_mfma_f32_32x32x2_f32)
//                       64x64 output tile per 256-thread workgroup, one 32x32 tile per wave,
//                       operands streamed straight to VGPRs (the f32 MFMA needs one VGPR per
//                       operand per lane), row norms accumulated from the same loads.
//  K1b knn_select_kernel one wave per row:
//                       1. per-lane sorted candidate lists over the D2 row (16-B loads);
//                       2. a 64-lane merge to kc = K-1+margin candidates, one DPP arg-min of
//                          the packed (d2, index) key per round;
//                       3. exact re-ranking with d^2 = sum_k (x_ik - x_jk)^2, eight candidates
//                          at a time (8-lane groups, DPP group sums) -- bitwise symmetric in
//                          (i, j) because both orders run the same lane mapping;
//                       4. the K-1 nearest by (exact d^2, index); self forced to rank 0 with
//                          distance 0 (the stand-in contract of SURVEY.md §8c);
//                       5. every valid pair (i -> j) is pushed onto j's reverse list (or the
//                          overflow list), which is how the symmetric union of GLL.py:197 is
//                          built without an n x n structure or a prefix sum.
#include <limits.h>

#include "gll_internal.h"

namespace gll {

// --------------------------------------------------------------------------------------
// K1a: Gram / squared-distance tile
// --------------------------------------------------------------------------------------
template <bool VEC>
__global__ __launch_bounds__(256) void gram_d2_kernel(const float* __restrict__ X, int n, int d,
                                                      float* __restrict__ D2, int ld,
                                                      int32_t* __restrict__ status,
                                                      int32_t* __restrict__ rev_cnt) {
    const int lane = lane_id();
    const int wave = threadIdx.x >> 6;
    const int r = lane & 31;   // A row / B column owned by this lane
    const int h = lane >> 5;   // k half: lane holds k = k0 + 4h + t, t = 0..3
    const int row0 = blockIdx.y * 64 + (wave >> 1) * 32;
    const int col0 = blockIdx.x * 64 + (wave & 1) * 32;
    // per-call reset of the counters the select kernel accumulates into
    {
        const int g = (blockIdx.y * gridDim.x + blockIdx.x) * 256 + threadIdx.x;
        if (g < GLL_ST_NWORDS) status[g] = 0;
        for (int q = g; q < n; q += gridDim.x * gridDim.y * 256) rev_cnt[q] = 0;
    }

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
// K1b: per-row selection + exact re-rank + reverse scatter
// --------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t pack_key(float d2, int j) {
    // d2 >= 0 after the clamp, so its IEEE bits order like the value; index breaks ties
    return (uint64_t(__float_as_uint(d2 > 0.f ? d2 : 0.f)) << 32) | uint32_t(j);
}

template <int KC>
__device__ __forceinline__ void list_insert(uint64_t (&key)[KC], uint64_t v) {
    // precondition: v < key[KC-1]; ascending order kept (keys are unique)
#pragma unroll
    for (int t = KC - 1; t > 0; --t) {
        const uint64_t prev = key[t - 1];
        key[t] = prev > v ? prev : (key[t] > v ? v : key[t]);
    }
    key[0] = key[0] > v ? v : key[0];
}

template <int KC>
__device__ __forceinline__ void list_pop(uint64_t (&key)[KC], bool pop) {
#pragma unroll
    for (int t = 0; t < KC - 1; ++t) key[t] = pop ? key[t + 1] : key[t];
    key[KC - 1] = pop ? ~0ull : key[KC - 1];
}

template <int KC, bool VEC>
__global__ __launch_bounds__(256) void knn_select_kernel(
    const float* __restrict__ D2, int ld, const float* __restrict__ X, int n, int d, int K,
    int kc, float eps_fixed, int auto_eps, int RCAP, int32_t* __restrict__ knn_idx,
    float* __restrict__ knn_d2, float* __restrict__ eps, int32_t* __restrict__ rev_cnt,
    int32_t* __restrict__ rev_idx, float* __restrict__ rev_d2, int32_t* __restrict__ ovf,
    int32_t* __restrict__ status, int32_t* __restrict__ status_pub) {
    const int lane = lane_id();
    const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (i >= n) return;  // whole wave

    // 1) per-lane scan of the row
    uint64_t key[KC];
#pragma unroll
    for (int t = 0; t < KC; ++t) key[t] = ~0ull;
    const float* row = D2 + size_t(i) * ld;
    for (int j0 = 4 * lane; j0 < n; j0 += 4 * kWave) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(row + j0);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int j = j0 + t;
            if (j < n && j != i && v[t] == v[t]) {   // NaN rows never enter
                const uint64_t kv = pack_key(v[t], j);
                if (kv < key[KC - 1]) list_insert<KC>(key, kv);
            }
        }
    }
    // 2) merge: round t hands the t-th smallest key to lane t
    uint64_t mine = ~0ull;
    for (int t = 0; t < kc; ++t) {
        const uint64_t best = wave_min_u64(key[0]);
        if (lane == t) mine = best;
        list_pop<KC>(key, best != ~0ull && key[0] == best);
    }
    const int ci = mine == ~0ull ? -1 : int(uint32_t(mine));
    // 3) exact squared distances, 8 candidates per pass (8 lanes each, across d)
    const int grp = lane >> 3, sub = lane & 7;
    const float* xi = X + size_t(i) * d;
    float ce = __builtin_inff();
    for (int p0 = 0; p0 < kc; p0 += 8) {
        const int j = __shfl(ci, p0 + grp < kc ? p0 + grp : 0);
        const bool live = p0 + grp < kc && j >= 0;
        const float* xj = X + size_t(live ? j : i) * d;
        float part = 0.f;
        for (int k = 4 * sub; k < d; k += 32) {
            const f32x4 a = load4<VEC>(xi, k, d);
            const f32x4 bb = load4<VEC>(xj, k, d);
            const f32x4 df = a - bb;
            part += df.x * df.x;
            part += df.y * df.y;
            part += df.z * df.z;
            part += df.w * df.w;
        }
        part = group8_sum(part);
#pragma unroll
        for (int g = 0; g < 8; ++g) {
            const float v = readlane_f(part, 8 * g);
            if (lane == p0 + g) ce = v;
        }
    }
    if (ci < 0) ce = __builtin_inff();
    // 4) rank the candidates by (exact d^2, index); keep the K-1 nearest
    const uint64_t myk = ci < 0 ? ~0ull : pack_key(ce, ci);
    int rank = 0;
    for (int u = 0; u < kc; ++u) {
        const uint32_t lo = __builtin_amdgcn_readlane(uint32_t(myk), u);
        const uint32_t hi = __builtin_amdgcn_readlane(uint32_t(myk >> 32), u);
        const uint64_t ku = (uint64_t(hi) << 32) | lo;
        rank += ku < myk ? 1 : 0;
    }
    const bool keep = lane < kc && ci >= 0 && rank < K - 1;
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
    // rows with fewer valid candidates (non-finite input) fall back to self at distance 0,
    // i.e. dropped edges (sparse.find drops zeros, GLL.py:198)
    const int nkeep = __popcll(__ballot(keep));
    if (lane >= nkeep && lane < K - 1) {
        oi[1 + lane] = i;
        od[1 + lane] = 0.f;
    }
    float ei = eps_fixed;
    if (auto_eps) {
        // eps_i = d(i, knn_ind[i, K-1])  (GLL.py:205)
        const float e = (keep && rank == K - 2) ? sqrtf(ce) : 0.f;
        ei = wave_sum_dpp(e);
    }
    if (lane == 0) {
        eps[i] = ei;
        if (!(ei >= 1e-10f)) atomicOr(&status_pub[GLL_ST_TINY_EPS], 1);  // GLL.py:240-241
    }
    // 5) reverse entry (ci, i) for every valid pair; zero distances never enter the graph
    if (keep && ce > 0.f) {
        const int pos = atomicAdd(&rev_cnt[ci], 1);
        if (pos < RCAP) {
            rev_idx[size_t(ci) * RCAP + pos] = i;
            rev_d2[size_t(ci) * RCAP + pos] = ce;
        } else {
            const int q = atomicAdd(&status[kStOvfCount], 1);
            ovf[3 * q + 0] = ci;
            ovf[3 * q + 1] = i;
            ovf[3 * q + 2] = __float_as_int(ce);
        }
    }
}

hipError_t launch_gram(const Layout& L, void* ws, const float* X, bool vec, hipStream_t s) {
    dim3 grid((L.n + 63) / 64, (L.n + 63) / 64);
    float* D2 = L.at<float>(ws, L.D2);
    int32_t* st = L.at<int32_t>(ws, L.status);
    int32_t* rc = L.at<int32_t>(ws, L.rev_cnt);
    prof_begin(GLL_K_GRAM, s);
    if (vec) gram_d2_kernel<true><<<grid, 256, 0, s>>>(X, L.n, L.d, D2, L.ldD, st, rc);
    else gram_d2_kernel<false><<<grid, 256, 0, s>>>(X, L.n, L.d, D2, L.ldD, st, rc);
    prof_end(GLL_K_GRAM, s);
    return hipGetLastError();
}

hipError_t launch_select(const Layout& L, void* ws, const float* X, float eps_fixed,
                         bool auto_eps, bool vec, int32_t* status_pub, hipStream_t s) {
    const int n = L.n, K = L.K;
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
    knn_select_kernel<KCV, V><<<grid, 256, 0, s>>>(                                            \
        L.at<float>(ws, L.D2), L.ldD, X, n, L.d, K, kc, eps_fixed, auto_eps ? 1 : 0, L.RCAP,    \
        L.at<int32_t>(ws, L.knn_idx), L.at<float>(ws, L.knn_d2), L.at<float>(ws, L.eps),       \
        L.at<int32_t>(ws, L.rev_cnt), L.at<int32_t>(ws, L.rev_idx), L.at<float>(ws, L.rev_d2), \
        L.at<int32_t>(ws, L.ovf), L.at<int32_t>(ws, L.status), status_pub)
    if (KC == 16) { if (vec) GLL_SEL(16, true); else GLL_SEL(16, false); }
    else if (KC == 32) { if (vec) GLL_SEL(32, true); else GLL_SEL(32, false); }
    else { if (vec) GLL_SEL(64, true); else GLL_SEL(64, false); }
#undef GLL_SEL
    prof_end(GLL_K_SELECT, s);
    return hipGetLastError();
}

}  // namespace gll
