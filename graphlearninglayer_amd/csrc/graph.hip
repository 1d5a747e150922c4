// graph.hip -- symmetric kNN graph in CSR + weights, degree and Laplace right-hand side.
//
// Replaces the scipy COO/CSR work of knn_sym_dist (/root/reference/GLL.py:192-238:
// coo->csr, symmetric max, sparse.find, W values) and csgraph.laplacian + the Luu/Lul
// split (GLL.py:29,37-38,48).  The union pattern is built without any n x n structure:
//   K2a pair_flag_kernel  one thread per directed kNN pair (i, j): valid (d > 0) and mutual
//                         (i in kNN(j)) flags; non-mutual pairs count a reverse entry for j.
//   K2b row_scan_kernel   single-workgroup exclusive scan of row lengths -> row_ptr.
//   K2c fill_kernel       forward entries at fixed slots, reverse entries via a row cursor.
//   K3  row_finalize_kernel  one wave per row: sort the row by column (deterministic order
//                         whatever the atomic fill order was), W_ij = exp(-4 d^2/(eps_i eps_j)),
//                         degree, split point (labeled columns first), Luu diagonal
//                         deg + tau, rhs = W_ul Y (= -Lul Y), P = [Y; .] and w = [0; .] rows.
// Self pairs and zero-distance pairs never enter the graph (sparse.find drops zeros).
#include "gll_internal.h"

namespace gll {

__global__ __launch_bounds__(256) void pair_flag_kernel(const int32_t* __restrict__ knn_idx,
                                                        const float* __restrict__ knn_d2, int n,
                                                        int K, uint8_t* __restrict__ flag,
                                                        int32_t* __restrict__ rev_cnt) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n * (K - 1)) return;
    const int i = g / (K - 1);
    const int t = 1 + g % (K - 1);
    const int j = knn_idx[size_t(i) * K + t];
    const float dd = knn_d2[size_t(i) * K + t];
    const bool valid = dd > 0.f && j != i && j >= 0 && j < n;
    bool mutual = false;
    if (valid) {
        const int32_t* lj = knn_idx + size_t(j) * K;
        for (int s = 1; s < K; ++s) mutual |= (lj[s] == i);
    }
    flag[size_t(i) * K + t] = uint8_t((valid ? 1 : 0) | (mutual ? 2 : 0));
    if (valid && !mutual) atomicAdd(&rev_cnt[j], 1);
}

__global__ __launch_bounds__(1024) void row_scan_kernel(const int32_t* __restrict__ fwd_cnt,
                                                        const int32_t* __restrict__ rev_cnt,
                                                        int n, int32_t* __restrict__ row_ptr) {
    __shared__ int wsum[16];
    const int tid = threadIdx.x;
    const int lane = tid & 63, w = tid >> 6;
    const int per = (n + 1023) / 1024;
    const int beg = min(tid * per, n), end = min(beg + per, n);
    int s = 0;
    for (int i = beg; i < end; ++i) s += fwd_cnt[i] + rev_cnt[i];
    int incl = s;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_up(incl, off);
        if (lane >= off) incl += v;
    }
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int excl = incl - s;
    for (int q = 0; q < w; ++q) excl += wsum[q];
    for (int i = beg; i < end; ++i) {
        row_ptr[i] = excl;
        excl += fwd_cnt[i] + rev_cnt[i];
    }
    if (tid == 1023) row_ptr[n] = excl;
}

__global__ __launch_bounds__(256) void fill_kernel(
    const int32_t* __restrict__ knn_idx, const float* __restrict__ knn_d2, int n, int K,
    const uint8_t* __restrict__ flag, const int32_t* __restrict__ row_ptr,
    const int32_t* __restrict__ fwd_cnt, int32_t* __restrict__ fill_cnt,
    int32_t* __restrict__ tmp_col, float* __restrict__ tmp_d2) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n * (K - 1)) return;
    const int i = g / (K - 1);
    const int t = 1 + g % (K - 1);
    const uint8_t* fi = flag + size_t(i) * K;
    const uint8_t f = fi[t];
    if (!(f & 1)) return;
    int pos = 0;
    for (int s = 1; s < t; ++s) pos += fi[s] & 1;
    const int j = knn_idx[size_t(i) * K + t];
    const float dd = knn_d2[size_t(i) * K + t];
    const int p = row_ptr[i] + pos;
    tmp_col[p] = j;
    tmp_d2[p] = dd;
    if (!(f & 2)) {  // j does not list i: reverse entry (j, i) goes after j's own entries
        const int q = row_ptr[j] + fwd_cnt[j] + atomicAdd(&fill_cnt[j], 1);
        tmp_col[q] = i;
        tmp_d2[q] = dd;
    }
}

template <typename TY>
__device__ __forceinline__ float yval(const TY* Y, int j, int C, int c) {
    return to_f32(Y[size_t(j) * C + c]);
}

constexpr int kRowChunk = 256;  // per-wave LDS staging of a sorted row (entries per pass)
constexpr int kMaxCPerLane = 4; // classes per lane in the rhs accumulation (C <= 256)

template <typename TY>
__global__ __launch_bounds__(256) void row_finalize_kernel(
    int n, int base, int C, float tau, const int32_t* __restrict__ row_ptr,
    const int32_t* __restrict__ tmp_col, const float* __restrict__ tmp_d2,
    const float* __restrict__ eps, const TY* __restrict__ Y, int32_t* __restrict__ col,
    float* __restrict__ w, float* __restrict__ d2e, float* __restrict__ deg,
    float* __restrict__ diag, float* __restrict__ rhs, float* __restrict__ P,
    float* __restrict__ Wadj, int32_t* __restrict__ ucnt) {
    __shared__ int s_col[4][kRowChunk];
    __shared__ float s_d2[4][kRowChunk];
    __shared__ float s_w[4][kRowChunk];
    const int lane = lane_id();
    const int wv = threadIdx.x >> 6;
    const int i = blockIdx.x * 4 + wv;
    if (i >= n) return;
    const int beg = row_ptr[i];
    const int L = row_ptr[i + 1] - beg;
    const float ei = eps[i];

    float dsum = 0.f;
    int nlab = 0;
    float racc[kMaxCPerLane];
#pragma unroll
    for (int q = 0; q < kMaxCPerLane; ++q) racc[q] = 0.f;
    bool labeled_done = false;

    for (int lo = 0; lo < L; lo += kRowChunk) {
        const int hi = min(L, lo + kRowChunk);
        // rank-scatter this chunk of sorted positions into LDS (columns are unique per row)
        for (int e = lane; e < L; e += kWave) {
            const int c = tmp_col[beg + e];
            int rank = 0;
            for (int u = 0; u < L; ++u) rank += tmp_col[beg + u] < c ? 1 : 0;
            if (rank >= lo && rank < hi) {
                s_col[wv][rank - lo] = c;
                s_d2[wv][rank - lo] = tmp_d2[beg + e];
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (int e = lo + lane; e < hi; e += kWave) {
            const int c = s_col[wv][e - lo];
            const float dd = s_d2[wv][e - lo];
            const float we = expf(-4.f * dd / (ei * eps[c]));   // GLL.py:216/233
            col[beg + e] = c;
            d2e[beg + e] = dd;
            w[beg + e] = we;
            s_w[wv][e - lo] = we;
            dsum += we;
            nlab += c < base ? 1 : 0;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // rhs_i = sum_{j < base} W_ij Y_j, labeled columns are the leading sorted entries
        if (i >= base && !labeled_done) {
            for (int e = lo; e < hi; ++e) {
                const int j = s_col[wv][e - lo];
                if (j >= base) {
                    labeled_done = true;
                    break;
                }
                const float we = s_w[wv][e - lo];
#pragma unroll
                for (int q = 0; q < kMaxCPerLane; ++q) {
                    const int c = lane + q * kWave;
                    if (c < C) racc[q] += we * yval(Y, j, C, c);
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    dsum = wave_sum(dsum);
    if (lane == 0) deg[i] = dsum;
#pragma unroll
    for (int q = 0; q < kMaxCPerLane; ++q) {
        const int c = lane + q * kWave;
        if (c < C) {
            if (i >= base) {
                rhs[size_t(i - base) * C + c] = racc[q];
            } else {
                P[size_t(i) * C + c] = yval(Y, i, C, c);
                Wadj[size_t(i) * C + c] = 0.f;
            }
        }
    }
    nlab = wave_sum_i(nlab);
    if (i >= base && lane == 0) {
        diag[i - base] = dsum + tau;   // Luu + tau I (GLL.py:48)
        ucnt[i - base] = L - nlab;     // the U block is the row's sorted suffix
    }
}

hipError_t launch_graph_build(const Layout& L, void* ws, hipStream_t s) {
    const int n = L.n, K = L.K;
    const int npairs = n * (K - 1);
    const int g = (npairs + 255) / 256;
    int32_t* knn_idx = L.at<int32_t>(ws, L.knn_idx);
    float* knn_d2 = L.at<float>(ws, L.knn_d2);
    uint8_t* flag = L.at<uint8_t>(ws, L.flag);
    prof_begin(GLL_K_MUTUAL, s);
    pair_flag_kernel<<<g, 256, 0, s>>>(knn_idx, knn_d2, n, K, flag, L.at<int32_t>(ws, L.rev_cnt));
    prof_end(GLL_K_MUTUAL, s);
    prof_begin(GLL_K_SCAN, s);
    row_scan_kernel<<<1, 1024, 0, s>>>(L.at<int32_t>(ws, L.fwd_cnt), L.at<int32_t>(ws, L.rev_cnt),
                                       n, L.at<int32_t>(ws, L.row_ptr));
    prof_end(GLL_K_SCAN, s);
    prof_begin(GLL_K_FILL, s);
    fill_kernel<<<g, 256, 0, s>>>(knn_idx, knn_d2, n, K, flag, L.at<int32_t>(ws, L.row_ptr),
                                  L.at<int32_t>(ws, L.fwd_cnt), L.at<int32_t>(ws, L.fill_cnt),
                                  L.at<int32_t>(ws, L.tmp_col), L.at<float>(ws, L.tmp_d2));
    prof_end(GLL_K_FILL, s);
    return hipGetLastError();
}

hipError_t launch_finalize(const Layout& L, void* ws, const void* Y, int y_dtype, float tau,
                           hipStream_t s) {
    if (L.C > kMaxCPerLane * kWave) return hipErrorInvalidValue;
    dim3 grid((L.n + 3) / 4);
#define GLL_FIN(T)                                                                             \
    row_finalize_kernel<T><<<grid, 256, 0, s>>>(                                               \
        L.n, L.base, L.C, tau, L.at<int32_t>(ws, L.row_ptr), L.at<int32_t>(ws, L.tmp_col),     \
        L.at<float>(ws, L.tmp_d2), L.at<float>(ws, L.eps), static_cast<const T*>(Y),           \
        L.at<int32_t>(ws, L.col), L.at<float>(ws, L.w), L.at<float>(ws, L.d2e),                \
        L.at<float>(ws, L.deg), L.at<float>(ws, L.diag), L.at<float>(ws, L.rhs),               \
        L.at<float>(ws, L.P), L.at<float>(ws, L.Wadj), L.at<int32_t>(ws, L.ucnt))
    prof_begin(GLL_K_FINALIZE, s);
    if (y_dtype == GLL_DT_F32) GLL_FIN(float);
    else if (y_dtype == GLL_DT_F64) GLL_FIN(double);
    else if (y_dtype == GLL_DT_I64) GLL_FIN(int64_t);
    else return hipErrorInvalidValue;
#undef GLL_FIN
    prof_end(GLL_K_FINALIZE, s);
    return hipGetLastError();
}

}  // namespace gll
