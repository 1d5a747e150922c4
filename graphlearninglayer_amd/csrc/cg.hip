// cg.hip -- Jacobi-preconditioned conjugate gradients on Luu (and on a general CSR).
//
// Replaces the SuperLU `spsolve(Luu, -Lul Y)` of the forward (/root/reference/GLL.py:53)
// and `spsolve(Luu, grad_output)` of the backward (GLL.py:93); the algorithm is the
// per-column masked CG of stable_conjgrad (GLL.py:247-276) with a Jacobi preconditioner
// (the reference's commented-out variant, GLL.py:55-64), WITHOUT its `p = r` aliasing
// quirk.  Each right-hand-side column is an independent system, so
// one workgroup owns one column: no inter-workgroup traffic, no host synchronisation, the
// iteration loop and the convergence test live on the device.
//
// Luu is never materialised: row u (graph row i = base + u) is
//     diag[u] * p_u - sum_{e in row i, col_e >= base} w_e * p_{col_e - base}
// over the sorted CSR of the symmetric kNN graph (labeled columns first, so the U block of
// a row is its tail [row_ptr[i] + split_i, row_ptr[i+1])).  When they fit, the vectors
// (x, r, p, Ap, M^-1) and the U-part of the CSR (cols, weights) are staged in LDS.
#include "gll_internal.h"

namespace gll {

template <int NT>
struct BlockRed {
    static constexpr int NW = NT / kWave;
    float* buf;   // 2 phases x 2 values x NW
    int phase = 0;
    __device__ __forceinline__ void sum2(float& a, float& b) {
        a = wave_sum(a);
        b = wave_sum(b);
        float* q = buf + phase * 2 * NW;
        phase ^= 1;
        if (lane_id() == 0) {
            q[threadIdx.x >> 6] = a;
            q[NW + (threadIdx.x >> 6)] = b;
        }
        __syncthreads();
        a = 0.f;
        b = 0.f;
#pragma unroll
        for (int w = 0; w < NW; ++w) {
            a += q[w];
            b += q[NW + w];
        }
    }
};

// Vectors live in LDS when vec_in_lds (else in the workspace); the U-part of the CSR is
// staged in LDS when it holds at most mat_cap entries (decided on the device: its size is
// only known after the graph build).
template <int NT, typename TB>
__global__ __launch_bounds__(NT) void cg_luu_kernel(
    int m, int C, int base, const int32_t* __restrict__ row_ptr, const int32_t* __restrict__ col,
    const float* __restrict__ wv, const float* __restrict__ diag, const TB* __restrict__ bsrc,
    double* __restrict__ out64, float* __restrict__ out32, float rtol, int max_iter,
    float* __restrict__ gvec, int vec_in_lds, int mat_cap, int32_t* __restrict__ st_nonconv,
    int32_t* __restrict__ st_iters) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int c = blockIdx.x;
    const int tid = threadIdx.x;
    BlockRed<NT> red{smem};
    float* vbase = smem + 4 * BlockRed<NT>::NW;
    if (!vec_in_lds) vbase = gvec + size_t(c) * 5 * m;
    float* X_ = vbase;
    float* R_ = vbase + m;
    float* P_ = vbase + 2 * m;
    float* A_ = vbase + 3 * m;
    float* M_ = vbase + 4 * m;
    // U-part of the CSR: positions [e0, e1) of the graph rows base..n-1
    const int e0 = row_ptr[base];
    const int e1 = row_ptr[base + m];
    const bool matl = (e1 - e0) <= mat_cap;
    int* lcol = reinterpret_cast<int*>(smem + 4 * BlockRed<NT>::NW + (vec_in_lds ? 5 * m : 0));
    float* lw = reinterpret_cast<float*>(lcol + (e1 - e0));
    if (matl) {
        for (int e = e0 + tid; e < e1; e += NT) {
            lcol[e - e0] = col[e] - base;
            lw[e - e0] = wv[e];
        }
    }
    // x0 = 0, r = b, z = M^-1 r, p = z
    float rz = 0.f, bb = 0.f;
    for (int u = tid; u < m; u += NT) {
        const float dg = diag[u];
        const float mi = dg > 0.f ? 1.f / dg : 0.f;
        const float bu = to_f32(bsrc[size_t(u) * C + c]);
        const float rb = mi > 0.f ? bu : 0.f;  // rows with zero diagonal are decoupled: x = 0
        X_[u] = 0.f;
        R_[u] = rb;
        M_[u] = mi;
        P_[u] = mi * rb;
        rz += rb * mi * rb;
        bb += rb * rb;
    }
    red.sum2(rz, bb);  // includes the barrier that publishes the LDS vectors/matrix
    const float tol2 = rtol * rtol * bb;
    int it = 0;
    bool conv = bb <= tol2 || bb == 0.f;
    while (!conv && it < max_iter) {
        ++it;
        // Ap and p.Ap
        float pap = 0.f, dummy = 0.f;
        for (int u = tid; u < m; u += NT) {
            const int i = base + u;
            const int rb0 = row_ptr[i], rb1 = row_ptr[i + 1];
            float acc = 0.f;
            if (matl) {
                // the U part is the tail of the sorted row; scan back from the end
                for (int e = rb1 - 1; e >= rb0; --e) {
                    const int j = lcol[e - e0];
                    if (j < 0) break;
                    acc += lw[e - e0] * P_[j];
                }
            } else {
                for (int e = rb1 - 1; e >= rb0; --e) {
                    const int j = col[e] - base;
                    if (j < 0) break;
                    acc += wv[e] * P_[j];
                }
            }
            const float pu = P_[u];
            const float ap = diag[u] * pu - acc;
            A_[u] = ap;
            pap += pu * ap;
        }
        red.sum2(pap, dummy);
        if (!(pap > 0.f)) break;  // breakdown (or NaN): stop, report non-convergence
        const float alpha = rz / pap;
        float rr = 0.f, rzn = 0.f;
        for (int u = tid; u < m; u += NT) {
            X_[u] += alpha * P_[u];
            const float ru = R_[u] - alpha * A_[u];
            R_[u] = ru;
            rr += ru * ru;
            rzn += ru * M_[u] * ru;
        }
        red.sum2(rr, rzn);
        if (rr <= tol2) {
            conv = true;
            break;
        }
        const float beta = rzn / rz;
        rz = rzn;
        for (int u = tid; u < m; u += NT) P_[u] = M_[u] * R_[u] + beta * P_[u];
        __syncthreads();
    }
    for (int u = tid; u < m; u += NT) {
        const float xu = X_[u];
        if (out64) out64[size_t(u) * C + c] = double(xu);
        if (out32) out32[size_t(u) * C + c] = xu;
    }
    if (tid == 0) {
        if (st_iters) atomicMax(st_iters, it);
        if (!conv && st_nonconv) atomicAdd(st_nonconv, 1);
    }
}

static constexpr size_t kLdsLimit = 160 * 1024;
static constexpr size_t kRedBytes = 4 * 16 * sizeof(float);

template <int NT, typename TB>
static hipError_t run_cg(const Layout& L, void* ws, const TB* b, double* out64, float* out32,
                         float rtol, int max_iter, int32_t* st_nonconv, int32_t* st_iters,
                         hipStream_t s) {
    const int m = L.m;
    const size_t vec_bytes = size_t(5) * m * sizeof(float);
    const bool vec_lds = kRedBytes + vec_bytes <= kLdsLimit;
    size_t lds = kRedBytes + (vec_lds ? vec_bytes : 0);
    // entries of the graph rows >= base: m(K-1) forward + at most n(K-1) reverse
    const int64_t eu_bound = int64_t(m + L.n) * (L.K - 1);
    int64_t cap = int64_t(kLdsLimit - lds) / 8;
    if (cap > eu_bound) cap = eu_bound;
    if (cap < 0) cap = 0;
    lds += size_t(cap) * 8;
    auto fn = cg_luu_kernel<NT, TB>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                        hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
    fn<<<L.C, NT, lds, s>>>(m, L.C, L.base, L.at<int32_t>(ws, L.row_ptr),
                            L.at<int32_t>(ws, L.col), L.at<float>(ws, L.w),
                            L.at<float>(ws, L.diag), b, out64, out32, rtol, max_iter,
                            L.at<float>(ws, L.cgv), vec_lds ? 1 : 0, int(cap), st_nonconv,
                            st_iters);
    return hipGetLastError();
}

template <typename TB>
static hipError_t cg_dispatch(const Layout& L, void* ws, const TB* b, double* out64,
                              float* out32, float rtol, int max_iter, int32_t* st_nonconv,
                              int32_t* st_iters, hipStream_t s) {
    if (L.m <= 2048)
        return run_cg<256, TB>(L, ws, b, out64, out32, rtol, max_iter, st_nonconv, st_iters, s);
    return run_cg<1024, TB>(L, ws, b, out64, out32, rtol, max_iter, st_nonconv, st_iters, s);
}

hipError_t launch_cg_luu(const Layout& L, void* ws, const void* b, int b_dtype, double* out64,
                         float* out32, float rtol, int max_iter, int32_t* st_nonconv,
                         int32_t* st_iters, hipStream_t s) {
    if (L.m <= 0) return hipSuccess;
    hipError_t e;
    prof_begin(GLL_K_CG, s);
    if (b_dtype == GLL_DT_F32)
        e = cg_dispatch(L, ws, static_cast<const float*>(b), out64, out32, rtol, max_iter,
                        st_nonconv, st_iters, s);
    else if (b_dtype == GLL_DT_F64)
        e = cg_dispatch(L, ws, static_cast<const double*>(b), out64, out32, rtol, max_iter,
                        st_nonconv, st_iters, s);
    else
        return hipErrorInvalidValue;
    prof_end(GLL_K_CG, s);
    return e;
}

// --------------------------------------------------------------------------------------
// General SPD CSR (stable_conjgrad replacement, absolute tolerance like GLL.py:259)
// --------------------------------------------------------------------------------------
template <int NT>
__global__ __launch_bounds__(NT) void cg_csr_kernel(int m, int C, const int32_t* __restrict__ rp,
                                                    const int32_t* __restrict__ col,
                                                    const float* __restrict__ val,
                                                    const float* __restrict__ b,
                                                    float* __restrict__ x, float atol,
                                                    int max_iter, float* __restrict__ gvec,
                                                    int vec_in_lds, int32_t* __restrict__ iters,
                                                    int32_t* __restrict__ nonconv) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int c = blockIdx.x;
    const int tid = threadIdx.x;
    BlockRed<NT> red{smem};
    float* vb = vec_in_lds ? smem + 4 * BlockRed<NT>::NW : gvec + size_t(c) * 5 * m;
    float *X_ = vb, *R_ = vb + m, *P_ = vb + 2 * m, *A_ = vb + 3 * m, *M_ = vb + 4 * m;
    float rz = 0.f, rr0 = 0.f;
    for (int u = tid; u < m; u += NT) {
        float dg = 0.f;
        for (int e = rp[u]; e < rp[u + 1]; ++e)
            if (col[e] == u) dg += val[e];
        const float mi = dg > 0.f ? 1.f / dg : 0.f;
        const float bu = b[size_t(u) * C + c];
        X_[u] = 0.f;
        R_[u] = bu;
        M_[u] = mi;
        P_[u] = mi * bu;
        rz += bu * mi * bu;
        rr0 += bu * bu;
    }
    red.sum2(rz, rr0);
    const float tol2 = atol * atol;
    int it = 0;
    bool conv = rr0 <= tol2;
    while (!conv && it < max_iter) {
        ++it;
        float pap = 0.f, dummy = 0.f;
        for (int u = tid; u < m; u += NT) {
            float acc = 0.f;
            for (int e = rp[u]; e < rp[u + 1]; ++e) acc += val[e] * P_[col[e]];
            A_[u] = acc;
            pap += P_[u] * acc;
        }
        red.sum2(pap, dummy);
        if (!(pap > 0.f)) break;
        const float alpha = rz / pap;
        float rr = 0.f, rzn = 0.f;
        for (int u = tid; u < m; u += NT) {
            X_[u] += alpha * P_[u];
            const float ru = R_[u] - alpha * A_[u];
            R_[u] = ru;
            rr += ru * ru;
            rzn += ru * M_[u] * ru;
        }
        red.sum2(rr, rzn);
        if (rr <= tol2) {
            conv = true;
            break;
        }
        const float beta = rzn / rz;
        rz = rzn;
        for (int u = tid; u < m; u += NT) P_[u] = M_[u] * R_[u] + beta * P_[u];
        __syncthreads();
    }
    for (int u = tid; u < m; u += NT) x[size_t(u) * C + c] = X_[u];
    if (tid == 0) {
        if (iters) atomicMax(iters, it);
        if (!conv && nonconv) atomicAdd(nonconv, 1);
    }
}

hipError_t launch_cg_csr(int m, int C, const int32_t* row_ptr, const int32_t* col,
                         const float* val, const float* b, float* x, float atol, int max_iter,
                         int32_t* iters, int32_t* nonconv, float* gvec, hipStream_t s) {
    const size_t vec_bytes = size_t(5) * m * sizeof(float);
    const bool vec_lds = kRedBytes + vec_bytes <= kLdsLimit;
    if (!vec_lds && gvec == nullptr) return hipErrorInvalidValue;
    const size_t lds = kRedBytes + (vec_lds ? vec_bytes : 0);
    auto fn = cg_csr_kernel<256>;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                        hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
    prof_begin(GLL_K_CG, s);
    fn<<<C, 256, lds, s>>>(m, C, row_ptr, col, val, b, x, atol, max_iter, gvec, vec_lds ? 1 : 0,
                           iters, nonconv);
    prof_end(GLL_K_CG, s);
    return hipGetLastError();
}

}  // namespace gll
