// gridcg.hip -- Jacobi-preconditioned CG over the whole GPU, for systems too large for one
// workgroup per right-hand side (the Luu solves of big graphs -- stress, utils.laplace at
// n ~ 60k -- and gll_cg_csr).  Same iteration as the per-column kernels of solve.hip and as
// stable_conjgrad (/root/reference/GLL.py:247-276, without its p-aliasing quirk): every
// column runs its own PCG with per-column step sizes, and a column is frozen once it meets
// its tolerance (GLL.py:258-268 masks alpha/beta the same way).
//
// cg_gv_kernel (round 3, the default): pipelined PCG (Ghysels & Vanroose 2014, Alg. 4) --
// ONE grid barrier per iteration.  Before the barrier a workgroup publishes m = M w for its
// rows together with its partial dot products (r,u), (w,u), (r,r); after it, the SpMV
// n = A m gathers the published m while the partials are summed, and every vector update is
// local.  The workgroup's slice of the matrix (column byte offsets and values) is staged in
// LDS once per solve, so an iteration reads nothing from global memory but the one published
// vector and the partials.  Rows past the LDS capacity read their entries from the CSR.
//
// cg_grid_classic_kernel (rounds 1-2): classic two-reduction PCG, two grid barriers per
// iteration, matrix entries and two vectors (z, p) gathered from global memory every iteration;
// kept for systems past the pipelined kernel's 512 rows per workgroup (m > 131,072) and the
// oversubscription test.  Cross-workgroup hand-offs in both: DESIGN.md §3.5.
//
// Dot products: each workgroup writes its partial sums, and after the barrier EVERY
// workgroup adds all partials in the same fixed order -- so every workgroup derives
// bitwise identical step sizes and convergence decisions (no broadcast, deterministic).
// Published vectors are m x Cp row-major fp32 in the workspace (a gathered row is Cp
// contiguous floats, Cp = C rounded up to 4).
#include <algorithm>
#include <cstdio>

#include "gll_internal.h"

namespace gll {

GLL_TRACE_UNIT(gridcg)

constexpr int kGT = 256;   // threads per workgroup
constexpr int kGCM = 16;   // columns held in registers (C <= kGCM)

// Luu of the padded graph rows: row u is graph row base+u, its U block the sorted suffix of
// length ucnt[u]; off-diagonal values -W, the diagonal deg + tau kept separately.
struct LuuRows {
    const int32_t* row_start;
    const int32_t* row_len;
    const int32_t* ucnt;
    const int32_t* col;
    const float* w;
    const float* diag;
    int base;
    __device__ int begin(int u) const { return row_start[base + u] + row_len[base + u] - ucnt[u]; }
    __device__ int end(int u) const { return row_start[base + u] + row_len[base + u]; }
    __device__ int column(int e) const { return col[e] - base; }
    __device__ float value(int e) const { return -w[e]; }
    __device__ float diagonal(int u) const { return diag[u]; }
    static constexpr bool kSeparateDiag = true;
};

// General CSR with the diagonal among the entries.
struct CsrRows {
    const int32_t* rp;
    const int32_t* col;
    const float* val;
    __device__ int begin(int u) const { return rp[u]; }
    __device__ int end(int u) const { return rp[u + 1]; }
    __device__ int column(int e) const { return col[e]; }
    __device__ float value(int e) const { return val[e]; }
    __device__ float diagonal(int u) const {
        float dg = 0.f;
        for (int e = rp[u]; e < rp[u + 1]; ++e)
            if (col[e] == u) dg += val[e];
        return dg;
    }
    static constexpr bool kSeparateDiag = false;
};

struct GridCgArgs {
    int m, C, Cp, max_iter;  // Cp: row stride of the published vectors (C rounded up to 4)
    float rtol, atol;        // per column: stop when ||r_c|| <= max(atol, rtol ||b_c||)
    const void* b;           // m x C right-hand sides, b_dtype
    int b_dtype;
    double* out64;           // m x C results (optional)
    float* out32;            // m x C results (optional)
    float* Pbuf;             // 2 x m x Cp: p of the previous iteration (double-buffered)
    float* Zbuf;             // m x Cp: z = M r of the previous iteration
    float* part;             // [G][3][kGCM] partial sums
    unsigned* sync;          // [0] arrivals, [1] failure word (zeroed before the launch)
    int rows_per_wg;
    int diag_fail;           // GLL_FLAG_DIAG_GRID_FAIL: inject a barrier failure (tests only)
    int32_t* st_iters;
    int32_t* st_nonconv;
    int32_t* st_failed;      // public GLL_ST_SOLVE_FAILED word
    int32_t* st_rescued;     // public GLL_ST_GRID_RESCUED word
    float* rescue;           // 5 m floats: the rescue solve's vectors
    int sync_zeroed;         // pipelined kernel: the sync words are known zero (no memset)
};

// Hand-off discipline: every byte another workgroup reads -- the published
// p / z rows and the partial sums -- is stored write-through (sc1) and loaded sc1 (16-B buffer
// accesses for the vectors), so the barrier needs neither an agent-scope release (a whole-L2
// write-back) nor an acquire (an L1/L2 invalidate); the writer drains its stores (vmcnt(0))
// before its relaxed arrival, the reader's loads are issued after its poll has seen the
// release.
__device__ __forceinline__ void st_shared(float* p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_shared(const float* p) {
    return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr int kSc1 = 16;   // buffer aux bit: sc1

// Grid barrier: one monotonic arrival counter (zeroed by a memset before the launch).  Every
// wave drains its sc1 stores, lane 0 arrives with a relaxed agent-scope add and polls the
// counter with sc1 loads and s_sleep; the spin is bounded, and a timeout raises the failure
// word every other poller also watches, so no wave can spin forever.
__device__ __forceinline__ bool grid_barrier(unsigned* sync, unsigned target, int* s_ok) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        int ok = 1;
        __hip_atomic_fetch_add(sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        const unsigned long long t0 = wall_ticks();
        while (__hip_atomic_load(sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if ((++spins & 1023u) == 0) {
                if (__hip_atomic_load(sync + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    ok = 0;
                    break;
                }
                if (wall_ticks() - t0 > kWaitTicks) {   // 1 s: a workgroup never arrived
                    __hip_atomic_store(sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = 0;
                    break;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler order only
        *s_ok = ok;
    }
    __syncthreads();
    return *s_ok != 0;
}

// Column-quad partial sums -> the workgroup's per-column partials (published sc1).  Lane li
// of every row group holds quad li; lanes with the same li are summed across the wave by
// xor shuffles, then across waves in LDS in wave order.
template <int LPR>
__device__ __forceinline__ void wg_partials(f32x4 v, float* red, float* out, int C) {
#pragma unroll
    for (int off = LPR; off < kWave; off <<= 1) {
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] += __shfl_xor(v[t], off);
    }
    const int lane = lane_id(), wv = threadIdx.x >> 6;
    if (lane < LPR && lane * 4 < kGCM) {
#pragma unroll
        for (int t = 0; t < 4; ++t) red[wv * kGCM + lane * 4 + t] = v[t];
    }
    __syncthreads();
    if (threadIdx.x < C) {
        float s = 0.f;
#pragma unroll
        for (int w = 0; w < kGT / kWave; ++w) s += red[w * kGCM + threadIdx.x];
        st_shared(out + threadIdx.x, s);
    }
    __syncthreads();
}

// After the barrier: every workgroup adds the G partials of slot `slot` in the same fixed
// tree (16 strided slices per column, then the slices in order) -> identical totals everywhere.
__device__ __forceinline__ void grid_totals(const float* part, int G, int slot, int C,
                                            float* red, float* tot) {
    const int c = threadIdx.x & 15, j = threadIdx.x >> 4;
    float s = 0.f;
    if (c < C) {
        const float* p = part + slot * kGCM + c;
#pragma unroll 4
        for (int g = j; g < G; g += 16) s += ld_shared(p + size_t(g) * 3 * kGCM);
    }
    red[j * 16 + c] = s;
    __syncthreads();
    if (threadIdx.x < C) {
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < 16; ++q) t += red[q * 16 + threadIdx.x];
        tot[threadIdx.x] = t;
    }
    __syncthreads();
}

__device__ __forceinline__ float rhs_at(const void* b, int dt, size_t i) {
    return dt == GLL_DT_F64 ? float(static_cast<const double*>(b)[i])
                            : static_cast<const float*>(b)[i];
}

// ---------------------------------------------------------------------------------------
// Rescue of a lost grid barrier.  The grid kernels need every workgroup resident at once; an
// ordinary launch does not promise that when other kernels hold CUs (a caller's side stream,
// an RCCL kernel that waits on a peer).  A barrier that times out (~1 s) no longer ends the
// solve with NaN: the first workgroup to see the failure claims the rescue word and solves
// every column alone -- per-column Jacobi PCG, the same iteration and stopping rule, vectors
// in the workspace (write-through sc1 accesses; one workgroup, so its barriers suffice) --
// while every other workgroup leaves without writing.  It depends on no other workgroup, so it
// always completes; the solve is slower (one CU) and GLL_ST_GRID_RESCUED counts it.
// ---------------------------------------------------------------------------------------
// The solution stores of the grid kernels: write-through (see rescued()).
__device__ __forceinline__ void st_out(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_out(float* p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NT>
__device__ float rescue_sum(float v, float* red) {
    v = wave_sum_dpp(v);
    __syncthreads();   // red is free (the previous sum was read)
    if (lane_id() == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < NT / kWave; ++w) t += red[w];
    return t;
}

template <class Mat, int NT>
__device__ void rescue_solve(const Mat& A, int m, int C, const void* b, int b_dtype, float rtol,
                             float atol, int max_iter, double* out64, float* out32,
                             float* scr /* 5 m floats */, int32_t* st_iters,
                             int32_t* st_nonconv, int32_t* st_rescued, unsigned* begun,
                             unsigned* finished) {
    __shared__ float red[NT / kWave];
    // every registered writer of the failed solve has counted out (bounded: they are resident
    // and past their last barrier) before this workgroup writes its first row
    auto wait_writers = [&]() {
        if (threadIdx.x == 0) {
            const unsigned long long t0 = wall_ticks();
            while (__hip_atomic_load(finished, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) !=
                       __hip_atomic_load(begun, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) &&
                   wall_ticks() - t0 < kWaitTicks)
                __builtin_amdgcn_s_sleep(2);
        }
        __syncthreads();
    };
    bool waited = false;
    float *X_ = scr, *R_ = scr + m, *P_ = scr + 2 * size_t(m), *Q_ = scr + 3 * size_t(m),
          *M_ = scr + 4 * size_t(m);
    int it_max = 0, nonconv = 0;
    for (int c = 0; c < C; ++c) {
        float rz = 0.f, bb = 0.f;
        for (int u = threadIdx.x; u < m; u += NT) {
            const float dg = A.diagonal(u);
            const float mi = dg > 0.f ? 1.f / dg : 0.f;
            const float bu = mi > 0.f ? rhs_at(b, b_dtype, size_t(u) * C + c) : 0.f;
            st_shared(X_ + u, 0.f);
            st_shared(R_ + u, bu);
            st_shared(M_ + u, mi);
            st_shared(P_ + u, mi * bu);
            rz += bu * mi * bu;
            bb += bu * bu;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        rz = rescue_sum<NT>(rz, red);
        bb = rescue_sum<NT>(bb, red);
        const float t = fmaxf(atol, rtol * sqrtf(bb));
        const float tol2 = t * t;
        bool conv = !(bb > tol2);
        int it = 0;
        while (!conv && it < max_iter) {
            ++it;
            float pq = 0.f;
            for (int u = threadIdx.x; u < m; u += NT) {
                float acc = Mat::kSeparateDiag ? A.diagonal(u) * ld_shared(P_ + u) : 0.f;
                for (int e = A.begin(u); e < A.end(u); ++e)
                    acc += A.value(e) * ld_shared(P_ + A.column(e));
                st_shared(Q_ + u, acc);
                pq += ld_shared(P_ + u) * acc;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            pq = rescue_sum<NT>(pq, red);
            if (!(pq > 0.f)) break;   // breakdown or NaN: non-converged
            const float alpha = rz / pq;
            float rr = 0.f, rzn = 0.f;
            for (int u = threadIdx.x; u < m; u += NT) {
                st_shared(X_ + u, ld_shared(X_ + u) + alpha * ld_shared(P_ + u));
                const float ru = ld_shared(R_ + u) - alpha * ld_shared(Q_ + u);
                st_shared(R_ + u, ru);
                rr += ru * ru;
                rzn += ru * ld_shared(M_ + u) * ru;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            rr = rescue_sum<NT>(rr, red);
            rzn = rescue_sum<NT>(rzn, red);
            if (rr <= tol2) {
                conv = true;
                break;
            }
            const float beta = rzn / rz;
            rz = rzn;
            for (int u = threadIdx.x; u < m; u += NT)
                st_shared(P_ + u, ld_shared(M_ + u) * ld_shared(R_ + u) + beta * ld_shared(P_ + u));
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        if (!waited) {
            wait_writers();
            waited = true;
        }
        for (int u = threadIdx.x; u < m; u += NT) {
            const float xv = ld_shared(X_ + u);
            if (out64) st_out(out64 + size_t(u) * C + c, double(xv));
            if (out32) st_out(out32 + size_t(u) * C + c, xv);
        }
        it_max = it > it_max ? it : it_max;
        nonconv += conv ? 0 : 1;
        __syncthreads();   // the next column reuses the vectors
    }
    if (threadIdx.x == 0) {
        if (st_iters) atomicMax(st_iters, it_max);
        if (st_nonconv && nonconv) atomicAdd(st_nonconv, nonconv);
        if (st_rescued) atomicAdd(st_rescued, 1);
    }
}

// After a grid kernel's loop: true when this workgroup must write nothing because a barrier
// failed (it rescued the solve, or another workgroup does).  A workgroup whose own barriers all
// completed can still be in that case: a late arrival completes the final barrier just after
// another workgroup timed out on it and claimed the rescue.  Writers register before they read
// the failure word (`begun`, a returning atomic at the coherence point, so the read is issued
// after it), write their rows write-through (sc1: no dirty copy in their XCD's L2 can be written
// back over the rescue later) and then count themselves out (`finished`; a writer that reads the
// failure word set counts out without writing).  The rescuer solves, then waits until every
// registered writer has counted out and writes every row: a writer registering after that saw
// the failure word (set before the rescuer claimed) and wrote nothing.  So U is the rescue
// solution alone, never a mix of two solves (advisor, round 5).
template <class Mat, int NT, class Args>
__device__ bool rescued(bool ok, unsigned* fail_word, unsigned* rescue_word, unsigned* begun,
                        unsigned* finished, const Mat& A, const Args& a, float* scr, int* s_flag) {
    if (ok) {
        if (threadIdx.x == 0) {
            (void)__hip_atomic_fetch_add(begun, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const bool failed =
                __hip_atomic_load(fail_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
            if (failed)
                (void)__hip_atomic_fetch_add(finished, 1u, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
            *s_flag = failed;
        }
        __syncthreads();
        return *s_flag != 0;
    }
    if (threadIdx.x == 0)
        *s_flag = __hip_atomic_fetch_add(rescue_word, 1u, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT) == 0u;
    __syncthreads();
    if (*s_flag)
        rescue_solve<Mat, NT>(A, a.m, a.C, a.b, a.b_dtype, a.rtol, a.atol, a.max_iter, a.out64,
                              a.out32, scr, a.st_iters, a.st_nonconv, a.st_rescued, begun,
                              finished);
    return true;
}

// A writer's end of the protocol above: its sc1 stores are performed, then it counts out.
__device__ __forceinline__ void writer_done(unsigned* finished) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        (void)__hip_atomic_fetch_add(finished, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ f32x4 quad_of(const float* s, int q) {
    return f32x4{s[4 * q], s[4 * q + 1], s[4 * q + 2], s[4 * q + 3]};
}

// Workgroup w owns rows [w R, (w+1) R).  A group of LPR lanes owns up to RPG of them (rows
// grp, grp + NG, ...); lane li of the group owns column quad li (columns 4li..4li+3) of those
// rows and keeps x, r, p, z, Minv for them in registers for the whole solve.  Phase A: the
// group's lanes split each row's entries, gather the published rows p_j = z_j + beta p_j
// (two 16-B sc1 loads per quad) and xor-reduce; phase B updates the owned quads.  Two grid
// barriers per iteration; only the published p / z rows and the partials cross workgroups.
template <class Mat, int LPR, int RPG>
__global__ __launch_bounds__(kGT) void cg_grid_classic_kernel(Mat A, GridCgArgs a) {
    GLL_TRACE_SCOPE(0);
    __shared__ float red[256];
    __shared__ float s_rz[kGCM], s_tol2[kGCM], s_alpha[kGCM], s_beta[kGCM], s_tot[3 * kGCM];
    __shared__ int s_active[kGCM];
    __shared__ int s_ok;
    constexpr int NG = kGT / LPR;
    const int m = a.m, C = a.C, Cp = a.Cp, NQ = (C + 3) >> 2;
    const int G = gridDim.x;
    const int r0 = blockIdx.x * a.rows_per_wg;
    const int r1 = min(m, r0 + a.rows_per_wg);
    const int li = threadIdx.x % LPR;
    const int grp = threadIdx.x / LPR;
    const bool qown = li < NQ;
    float* mypart = a.part + size_t(blockIdx.x) * 3 * kGCM;
    const int vbytes = m * Cp * 4;
    const __amdgpu_buffer_rsrc_t rz_ = __builtin_amdgcn_make_buffer_rsrc(a.Zbuf, 0, vbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rp0 = __builtin_amdgcn_make_buffer_rsrc(a.Pbuf, 0, vbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rp1 =
        __builtin_amdgcn_make_buffer_rsrc(a.Pbuf + size_t(m) * Cp, 0, vbytes, 0x00020000);
    unsigned bar = 0;
    bool ok = true;

    f32x4 x[RPG], r[RPG], p[RPG], z[RPG], q[RPG];
    float mi[RPG], dg[RPG];
    // ---- setup: x = 0, r = b (decoupled rows: 0), z = M r, p = 0 (the first p is z);
    //      publish z and p(= 0); partial (r, z), (b, b)
    {
        f32x4 prz = {0.f, 0.f, 0.f, 0.f}, pbb = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < RPG; ++k) {
            const int u = r0 + grp + k * NG;
            x[k] = r[k] = p[k] = z[k] = q[k] = f32x4{0.f, 0.f, 0.f, 0.f};
            mi[k] = dg[k] = 0.f;
            if (u < r1) {
                dg[k] = A.diagonal(u);
                mi[k] = dg[k] > 0.f ? 1.f / dg[k] : 0.f;
                if (qown) {
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const int c = 4 * li + t;
                        const float bu = c < C ? rhs_at(a.b, a.b_dtype, size_t(u) * C + c) : 0.f;
                        r[k][t] = mi[k] > 0.f ? bu : 0.f;
                    }
                    z[k] = mi[k] * r[k];
                    prz += r[k] * z[k];
                    pbb += r[k] * r[k];
                    const int off = (u * Cp + 4 * li) * 4;
                    __builtin_amdgcn_raw_buffer_store_b128(z[k], rz_, off, 0, kSc1);
                    __builtin_amdgcn_raw_buffer_store_b128(p[k], rp1, off, 0, kSc1);
                }
            }
        }
        // slots 2 / 1: phase A of the first iteration writes slot 0 while slower
        // workgroups may still be summing these; slots 1-2 are next written after barrier A
        wg_partials<LPR>(prz, red, mypart + 2 * kGCM, C);
        wg_partials<LPR>(pbb, red, mypart + 1 * kGCM, C);
    }
    ok = grid_barrier(a.sync, (++bar) * G, &s_ok);
    grid_totals(a.part, G, 2, C, red, s_tot);
    grid_totals(a.part, G, 1, C, red, s_tot + kGCM);
    if (threadIdx.x < kGCM) {
        const int c = threadIdx.x;
        const float bb = c < C ? s_tot[kGCM + c] : 0.f;
        const float t = fmaxf(a.atol, a.rtol * sqrtf(bb));
        s_tol2[c] = t * t;
        s_rz[c] = c < C ? s_tot[c] : 0.f;
        s_active[c] = (c < C && bb > s_tol2[c]) ? 1 : 0;
        s_beta[c] = 0.f;
        s_alpha[c] = 0.f;
    }
    __syncthreads();
    int any = 0;
    for (int c = 0; c < C; ++c) any |= s_active[c];
    int it = 0;
    GLL_TRACE_PT(0);
    while (ok && any && it < a.max_iter) {
        ++it;
        const __amdgpu_buffer_rsrc_t prd = (it & 1) ? rp1 : rp0;   // p of iteration it-1
        const __amdgpu_buffer_rsrc_t pwr = (it & 1) ? rp0 : rp1;   // p of iteration it
        // ---- A: p = z + beta p (owned quads, published), q = A p, partial (p, q)
        {
            f32x4 bq[kGCM / 4];
#pragma unroll
            for (int qq = 0; qq < kGCM / 4; ++qq) bq[qq] = quad_of(s_beta, qq);
            const f32x4 bown = quad_of(s_beta, li < kGCM / 4 ? li : 0);
            f32x4 ppq = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < RPG; ++k) {
                const int u = r0 + grp + k * NG;
                if (u >= r1) continue;
                if (qown) {
                    p[k] = z[k] + bown * p[k];
                    __builtin_amdgcn_raw_buffer_store_b128(p[k], pwr, (u * Cp + 4 * li) * 4, 0,
                                                           kSc1);
                }
                f32x4 acc[kGCM / 4];
#pragma unroll
                for (int qq = 0; qq < kGCM / 4; ++qq) acc[qq] = f32x4{0.f, 0.f, 0.f, 0.f};
                const int e0 = A.begin(u), e1 = A.end(u);
                // entries in chunks of 4 per lane: index/value loads first, then every
                // gather of the chunk in flight together (2 memory round trips per chunk)
                for (int eb = e0 + li; eb < e1; eb += 4 * LPR) {
                    int off[4];
                    float vv[4];
#pragma unroll
                    for (int t = 0; t < 4; ++t) {
                        const int e = eb + t * LPR;
                        const bool live = e < e1;
                        const int ec = live ? e : eb;
                        off[t] = A.column(ec) * Cp * 4;
                        vv[t] = live ? A.value(ec) : 0.f;
                    }
#pragma unroll
                    for (int qq = 0; qq < kGCM / 4; ++qq) {
                        if (qq < NQ) {
                            f32x4 zj[4], pj[4];
#pragma unroll
                            for (int t = 0; t < 4; ++t) {
                                zj[t] = __builtin_amdgcn_raw_buffer_load_b128(rz_, off[t] + 16 * qq, 0, kSc1);
                                pj[t] = __builtin_amdgcn_raw_buffer_load_b128(prd, off[t] + 16 * qq, 0, kSc1);
                            }
#pragma unroll
                            for (int t = 0; t < 4; ++t) acc[qq] += vv[t] * (zj[t] + bq[qq] * pj[t]);
                        }
                    }
                }
#pragma unroll
                for (int qq = 0; qq < kGCM / 4; ++qq) {
#pragma unroll
                    for (int off = LPR / 2; off > 0; off >>= 1) {
#pragma unroll
                        for (int t = 0; t < 4; ++t) acc[qq][t] += __shfl_xor(acc[qq][t], off);
                    }
                }
                f32x4 mine = acc[0];
#pragma unroll
                for (int qq = 1; qq < kGCM / 4; ++qq) mine = li == qq ? acc[qq] : mine;
                q[k] = Mat::kSeparateDiag ? dg[k] * p[k] + mine : mine;
                if (qown) ppq += p[k] * q[k];
            }
            if (it == 1) GLL_TRACE_PT(2);
            wg_partials<LPR>(qown ? ppq : f32x4{0.f, 0.f, 0.f, 0.f}, red, mypart + 0 * kGCM, C);
        }
        ok = grid_barrier(a.sync, (++bar) * G, &s_ok);
        if (a.diag_fail && it == 2) ok = false;   // injected failure (uniform over the grid)
        if (it == 1) GLL_TRACE_PT(3);
        if (!ok) break;
        grid_totals(a.part, G, 0, C, red, s_tot);
        if (threadIdx.x < kGCM) {   // padding columns C..15 stay inactive: alpha = 0
            const int c = threadIdx.x;
            const float pq = c < C ? s_tot[c] : 0.f;
            int act = s_active[c];
            if (act == 1 && !(pq > 0.f)) act = 2;   // breakdown / NaN: stops, not converged
            s_active[c] = act;
            s_alpha[c] = act == 1 ? s_rz[c] / pq : 0.f;
        }
        __syncthreads();
        // ---- B: x += a p, r -= a q, z = M r (owned quads, z published), partial (r,r), (r,z)
        {
            const f32x4 al = quad_of(s_alpha, li < kGCM / 4 ? li : 0);
            f32x4 prr = {0.f, 0.f, 0.f, 0.f}, prz = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int k = 0; k < RPG; ++k) {
                const int u = r0 + grp + k * NG;
                if (u >= r1 || !qown) continue;
                x[k] += al * p[k];
                r[k] -= al * q[k];
                z[k] = mi[k] * r[k];
                prr += r[k] * r[k];
                prz += r[k] * z[k];
                __builtin_amdgcn_raw_buffer_store_b128(z[k], rz_, (u * Cp + 4 * li) * 4, 0, kSc1);
            }
            if (it == 1) GLL_TRACE_PT(4);
            wg_partials<LPR>(prr, red, mypart + 1 * kGCM, C);
            wg_partials<LPR>(prz, red, mypart + 2 * kGCM, C);
        }
        ok = grid_barrier(a.sync, (++bar) * G, &s_ok);
        if (it == 1) GLL_TRACE_PT(5);
        if (!ok) break;
        grid_totals(a.part, G, 1, C, red, s_tot + kGCM);
        grid_totals(a.part, G, 2, C, red, s_tot + 2 * kGCM);
        if (threadIdx.x < kGCM) {   // padding columns: beta = 0
            const int c = threadIdx.x;
            int act = s_active[c];
            const float rr = c < C ? s_tot[kGCM + c] : 0.f;
            const float rzn = c < C ? s_tot[2 * kGCM + c] : 0.f;
            if (act == 1 && rr <= s_tol2[c]) act = 0;   // converged
            s_beta[c] = act == 1 ? rzn / s_rz[c] : 0.f;
            if (act == 1) s_rz[c] = rzn;
            s_active[c] = act;
        }
        __syncthreads();
        any = 0;
        for (int c = 0; c < C; ++c) any |= (s_active[c] == 1);
        if (it == 1) GLL_TRACE_PT(6);
    }
    GLL_TRACE_PT(1);
    // a failed grid barrier (a workgroup never arrived within ~1 s): one workgroup solves the
    // system alone (rescue_solve), the others write nothing
    if (rescued<Mat, kGT>(ok, a.sync + 1, a.sync + 2, a.sync + 3, a.sync + 4, A, a, a.rescue,
                          &s_ok))
        return;
#pragma unroll
    for (int k = 0; k < RPG; ++k) {
        const int u = r0 + grp + k * NG;
        if (u >= r1 || !qown) continue;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int c = 4 * li + t;
            if (c < C) {
                const size_t i = size_t(u) * C + c;
                if (a.out64) st_out(a.out64 + i, double(x[k][t]));
                if (a.out32) st_out(a.out32 + i, x[k][t]);
            }
        }
    }
    writer_done(a.sync + 4);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        int nonconv = 0;
        for (int c = 0; c < C; ++c) nonconv += s_active[c] != 0 ? 1 : 0;
        if (a.st_iters) atomicMax(a.st_iters, it);
        if (a.st_nonconv && nonconv) atomicAdd(a.st_nonconv, nonconv);
    }
}

// ---------------------------------------------------------------------------------------
// Pipelined whole-GPU PCG (cg_gv_kernel)
// ---------------------------------------------------------------------------------------
constexpr int kMaxG = 256;            // workgroups of one pipelined solve (<= one per CU)
constexpr int kGvMaxRows = 512;       // rows per workgroup: NG x RPG <= 64 x 8
constexpr int kSyncLine = 32;         // words per sync word (one 128-B line each)
// sync lines: [0, 8) group arrival counters, 8 top counter, 9 failure, 10 rescue, [11, 19)
// release words (one per group), 19 exit counter, 20 / 21 writers registered / counted out
// (rescued())
#ifndef GLL_GV_GROUPS
#define GLL_GV_GROUPS 8
#endif
constexpr int kGvGroups = GLL_GV_GROUPS;   // arrival groups of the two-level barrier
constexpr int kSyncTop = kGvGroups, kSyncFail = kGvGroups + 1, kSyncRescue = kGvGroups + 2,
              kSyncRel = kGvGroups + 3, kSyncExit = 2 * kGvGroups + 3,
              kSyncBegun = 2 * kGvGroups + 4, kSyncFinished = 2 * kGvGroups + 5;
constexpr int kSyncWords = (2 * kGvGroups + 6) * kSyncLine;
static_assert(kSyncWords <= kGridSyncWords, "gll_internal.h kGridSyncWords (row_build zeroes them)");

struct GvArgs {
    int m, C, Cp, NQ, PW, max_iter;   // PW: partial floats per workgroup (32 or 64)
    float rtol, atol;                 // per column: stop when ||r_c|| <= max(atol, rtol ||b_c||)
    const void* b;                    // m x C right-hand sides, b_dtype
    int b_dtype;
    double* out64;                    // m x C results (optional)
    float* out32;                     // m x C results (optional)
    float* V;                         // [2][m][Cp] published vectors (u0, then m_i), by parity
    float* part;                      // [2][kMaxG][PW] partial sums, by parity
    unsigned* sync;                   // kSyncWords: zero at launch (gv_exit leaves them so)
    int rows_per_wg;
    int lds_cap;                      // matrix entries the dynamic LDS slice holds
    int hier;                         // two-level barrier (8 counters, then one)
    int diag_fail;                    // GLL_FLAG_DIAG_GRID_FAIL (tests only)
    int32_t* st_iters;
    int32_t* st_nonconv;
    int32_t* st_failed;
    int32_t* st_rescued;
    float* rescue;                    // 5 m floats: the rescue solve's vectors
};

// Grid barrier of the pipelined kernel.  Every wave drains its sc1 stores (asm vmcnt(0): the
// compiler does not count the buffer stores' completion by itself), the workgroup meets, and
// thread 0 arrives (relaxed agent-scope atomics, performed at the memory side):
//  - hier: an add to arrival counter (block % 8) whose returned value tells the group's last
//    arriver, which alone adds to the top counter (8 arrivals per epoch);
//  - flat: an add to the top counter (G arrivals per epoch).
// The arrival that completes the top counter writes the epoch into the 8 release words, and
// every workgroup polls its group's release word (sc1 loads, s_sleep): no poller reads a line
// that atomics land on -- round 3 polled the top counter itself, 256 pollers on the line the
// last arrivals were adding to, and the release came ~2.2 us after the last arrival
// (profiles/r04j_gv_trace.txt).  Placement-independent (the groups are block-index classes;
// they coincide with XCDs only for speed).  The spin is bounded and a timeout raises the
// failure word every poller also watches.  Monotonic: epoch e waits for e x arrivals.
__device__ __forceinline__ bool gv_barrier(unsigned* sync, unsigned epoch, int G, int hier,
                                           int* s_ok) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned* top = sync + kSyncTop * kSyncLine;
        unsigned* fail = sync + kSyncFail * kSyncLine;
        unsigned* rel = sync + kSyncRel * kSyncLine;
        const int ng = G < kGvGroups ? G : kGvGroups;
        const int g = int(blockIdx.x) % ng;
        bool last;
        if (hier) {
            const unsigned gs = unsigned((G - g + ng - 1) / ng);
            const unsigned old = __hip_atomic_fetch_add(sync + g * kSyncLine, 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
            last = old + 1u == epoch * gs &&
                   __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u ==
                       epoch * unsigned(ng);
        } else {
            last = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u ==
                   epoch * unsigned(G);
        }
        if (last)
            for (int q = 0; q < ng; ++q)
                __hip_atomic_store(rel + q * kSyncLine, epoch, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        int ok = 1;
        unsigned spins = 0;
        const unsigned long long t0 = wall_ticks();
        while (__hip_atomic_load(rel + g * kSyncLine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
               epoch) {
            __builtin_amdgcn_s_sleep(1);
            if ((++spins & 1023u) == 0) {
                if (__hip_atomic_load(fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    ok = 0;
                    break;
                }
                if (wall_ticks() - t0 > kWaitTicks) {   // 1 s: a workgroup never arrived
                    __hip_atomic_store(fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = 0;
                    break;
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler order only
        *s_ok = ok;
    }
    __syncthreads();
    return *s_ok != 0;
}

// End of a pipelined solve: every workgroup counts out, and the last one returns the sync words
// to zero (every other workgroup of the grid has left, rescued or not), so the next solve on
// this workspace starts from zero without a memset launch (row_build zeroes them before a
// forward; gll_cg_csr's caller workspace still gets a memset).
__device__ __forceinline__ void gv_exit(unsigned* sync, int G, int* s_flag) {
    __syncthreads();
    if (threadIdx.x == 0)
        *s_flag = __hip_atomic_fetch_add(sync + kSyncExit * kSyncLine, 1u, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT) == unsigned(G - 1);
    __syncthreads();
    if (*s_flag)
        for (int t = threadIdx.x; t < kSyncWords; t += blockDim.x)
            __hip_atomic_store(sync + t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sum over each aligned group of LPR lanes, result in every lane of the group (DPP: quad
// butterflies, then the half-row and row mirrors).  Fixed order -> deterministic.
template <int LPR>
__device__ __forceinline__ float group_sum(float v) {
    v = dpp_add<0xB1, 0xf>(v);                       // quad_perm [1,0,3,2]
    v = dpp_add<0x4E, 0xf>(v);                       // quad_perm [2,3,0,1]
    if constexpr (LPR >= 8) v = dpp_add<0x141, 0xf>(v);   // row_half_mirror
    if constexpr (LPR >= 16) v = dpp_add<0x140, 0xf>(v);  // row_mirror
    return v;
}

__device__ __forceinline__ int wave_excl_scan(int v, int* total) {
    int x = v;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const int y = __shfl_up(x, off);
        if (lane_id() >= off) x += y;
    }
    *total = __shfl(x, kWave - 1);
    return x - v;
}

constexpr int kOob = 0x7FFFFFF0;   // buffer offset past any num_records: the load returns 0

// Workgroup w owns rows [w R, (w+1) R).  A group of LPR lanes owns up to RPG of them (local
// rows grp, grp + NG, ...); lane li of the group owns column quad li (columns 4li..4li+3) of
// those rows and keeps x, r, u, w, p, s, q, z for them in registers for the whole solve.
// The group's lanes split each row's entries for the gathers and sum them by DPP.
// MODE 0: pipelined PCG (Ghysels-Vanroose), one grid barrier per iteration.  MODE 1:
// Chronopoulos-Gear single-reduction PCG on the same machinery, two barriers per iteration
// (u published, then the partials): its recurrences keep fp32 attainable accuracy close to
// classic PCG's, where GV's drift on ill-conditioned systems -- utils.laplace's tau = 1e-8 at
// 60,250 points took 303 GV iterations against 92 (profiles/r03c_laplace_probe.txt).
template <class Mat, int NT, int LPR, int RPG, int MODE>
__global__ __launch_bounds__(NT) void cg_gv_kernel(Mat A, GvArgs a) {
    GLL_TRACE_SCOPE(1);
    extern __shared__ __attribute__((aligned(16))) int2 s_ent[];   // (byte offset, value bits)
    __shared__ int s_len[kGvMaxRows];
    __shared__ float s_wp[NT / kWave][64];        // per-wave partials, slots [0,3C)
    __shared__ f32x4 s_red[NT / kWave][16];       // per-wave sums of the loaded partials
    __shared__ int s_ok;
    constexpr int NG = NT / LPR;
    constexpr int NW = NT / kWave;
    constexpr int JP = kMaxG * 16 / NT;   // partial float4 loads per thread
    const int m = a.m, C = a.C, Cp = a.Cp, NQ = a.NQ, PW = a.PW;
    const int G = gridDim.x;
    const int r0 = blockIdx.x * a.rows_per_wg;
    const int r1 = min(m, r0 + a.rows_per_wg);
    const int li = threadIdx.x % LPR;
    const int grp = threadIdx.x / LPR;
    const int wv = threadIdx.x >> 6, lane = lane_id();
    const bool qown = li < NQ;
    const int rowB = Cp * 4;
    const int vbytes = m * rowB;
    const __amdgpu_buffer_rsrc_t rv0 = __builtin_amdgcn_make_buffer_rsrc(a.V, 0, vbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rv1 =
        __builtin_amdgcn_make_buffer_rsrc(a.V + size_t(m) * Cp, 0, vbytes, 0x00020000);
    const int pbytes = G * PW * 4;
    const __amdgpu_buffer_rsrc_t rpt0 = __builtin_amdgcn_make_buffer_rsrc(a.part, 0, pbytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rpt1 =
        __builtin_amdgcn_make_buffer_rsrc(a.part + size_t(kMaxG) * PW, 0, pbytes, 0x00020000);

    // ---- the workgroup's matrix slice -> LDS (once per solve)
    int len[RPG], off[RPG], gb[RPG];
#pragma unroll
    for (int k = 0; k < RPG; ++k) {
        const int lr = grp + k * NG;
        const int u = r0 + lr;
        len[k] = 0;
        gb[k] = 0;
        if (u < r1) {
            gb[k] = A.begin(u);
            len[k] = A.end(u) - gb[k];
        }
        if (li == 0) s_len[lr] = len[k];
    }
    for (int t = threadIdx.x; t < 64; t += NT)
        for (int w = 0; w < NW; ++w) s_wp[w][t] = 0.f;
    __syncthreads();
    if (threadIdx.x < kWave) {   // exclusive scan of the row lengths (wave 0)
        int carry = 0;
        for (int c0 = 0; c0 < NG * RPG; c0 += kWave) {
            const int v = s_len[c0 + lane];
            int tot;
            const int ex = wave_excl_scan(v, &tot);
            s_len[c0 + lane] = carry + ex;
            carry += tot;
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < RPG; ++k) {
        off[k] = s_len[grp + k * NG];
        for (int e = li; e < len[k]; e += LPR) {
            const int slot = off[k] + e;
            if (slot < a.lds_cap)
                s_ent[slot] = int2{A.column(gb[k] + e) * rowB,
                                   __builtin_bit_cast(int, A.value(gb[k] + e))};
        }
    }

    // n = A v over the owned rows: lane li gathers entries li, li + LPR, ... (chunks of CH per
    // lane, every gather of a chunk in flight together), the group sums by DPP, lane li keeps
    // quad li.  Dead entries load from an out-of-range offset (the buffer returns 0).
    // 256 threads: a row of up to 8 LPR entries in one round of gathers (the barrier waits for
    // the workgroup with the longest rows: at stress, 4 per lane left hub rows a second round
    // trip, and iteration 3's arrivals spread over 1.2 us, profiles/r04l_gv_trace.txt); 16 waves:
    // fewer gathers per lane, no spills
    constexpr int CH = NT >= 1024 ? 2 : 8;
    auto spmv = [&](int k, __amdgpu_buffer_rsrc_t rv) -> f32x4 {
        f32x4 acc[kGCM / 4];
#pragma unroll
        for (int qq = 0; qq < kGCM / 4; ++qq) acc[qq] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int eb = li; eb < len[k]; eb += CH * LPR) {
            int co[CH];
            float vv[CH];
#pragma unroll
            for (int t = 0; t < CH; ++t) {
                const int e = eb + t * LPR;
                int2 en = int2{kOob, 0};
                if (e < len[k]) {
                    const int slot = off[k] + e;
                    en = slot < a.lds_cap ? s_ent[slot]
                                          : int2{A.column(gb[k] + e) * rowB,
                                                 __builtin_bit_cast(int, A.value(gb[k] + e))};
                }
                co[t] = en.x;
                vv[t] = __builtin_bit_cast(float, en.y);
            }
#pragma unroll
            for (int qq = 0; qq < kGCM / 4; ++qq) {
                if (qq < NQ) {
                    f32x4 g[CH];
#pragma unroll
                    for (int t = 0; t < CH; ++t)
                        g[t] = __builtin_amdgcn_raw_buffer_load_b128(rv, co[t] + 16 * qq, 0, kSc1);
#pragma unroll
                    for (int t = 0; t < CH; ++t) acc[qq] += vv[t] * g[t];
                }
            }
        }
        f32x4 mine = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int qq = 0; qq < kGCM / 4; ++qq) {
            if (qq < NQ) {
#pragma unroll
                for (int t = 0; t < 4; ++t) acc[qq][t] = group_sum<LPR>(acc[qq][t]);
                mine = li == qq ? acc[qq] : mine;
            }
        }
        return mine;
    };

    // ---- setup: x = 0, r = b (decoupled rows: 0), u = M r published for w = A u
    f32x4 x[RPG], r[RPG], u[RPG], w[RPG], p[RPG], s[RPG], q[RPG], z[RPG];
    float mi[RPG], dg[RPG];
#pragma unroll
    for (int k = 0; k < RPG; ++k) {
        const int uu = r0 + grp + k * NG;
        x[k] = r[k] = u[k] = w[k] = p[k] = s[k] = q[k] = z[k] = f32x4{0.f, 0.f, 0.f, 0.f};
        mi[k] = dg[k] = 0.f;
        if (uu < r1) {
            dg[k] = A.diagonal(uu);
            mi[k] = dg[k] > 0.f ? 1.f / dg[k] : 0.f;
            if (qown) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int c = 4 * li + t;
                    const float bu = c < C ? rhs_at(a.b, a.b_dtype, size_t(uu) * C + c) : 0.f;
                    r[k][t] = mi[k] > 0.f ? bu : 0.f;
                }
                u[k] = mi[k] * r[k];
                __builtin_amdgcn_raw_buffer_store_b128(u[k], rv0, uu * rowB + 16 * li, 0, kSc1);
            }
        }
    }
    // per-column step-size state, lane c of EVERY wave for column c (the waves compute it
    // redundantly from the same sums in the same order: identical everywhere, no broadcast)
    int act_c = lane < C ? 1 : 0;   // 1 active, 0 converged, 2 broken down
    float gold_c = 1.f, aold_c = 1.f, tol2_c = 0.f;
    unsigned epoch = 0;
    bool ok = gv_barrier(a.sync, ++epoch, G, a.hier, &s_ok);
    if constexpr (MODE == 0) {
#pragma unroll
        for (int k = 0; k < RPG; ++k) {
            const int uu = r0 + grp + k * NG;
            if (uu < r1) {
                const f32x4 o = spmv(k, rv0);
                w[k] = Mat::kSeparateDiag ? dg[k] * u[k] + o : o;
            }
        }
    }

    int it = 0;
    GLL_TRACE_PT(8);
    // trace build: block 0's checkpoints of iteration 3 (words 11-18; tools/gv_trace.py)
#ifdef GLL_TRACE
    // ... and every workgroup's arrival at / release from iteration 3's barrier (g_wg[0, 8192))
#define GLL_GV_WG(slot)                                                                     \
    do {                                                                                    \
        if (it == 3 && threadIdx.x == 0 && blockIdx.x < 4096)                               \
            g_wg[(slot) * 4096 + blockIdx.x] = __builtin_amdgcn_s_memrealtime();            \
    } while (0)
#else
#define GLL_GV_WG(slot) do {} while (0)
#endif
#define GLL_GV_PT(i)                                 \
    do {                                             \
        if (it == 3) GLL_TRACE_PT(i);                \
        if (it == 4 && (i) == 11) GLL_TRACE_PT(18);  \
        if ((i) == 12) GLL_GV_WG(0);                 \
        if ((i) == 13) GLL_GV_WG(1);                 \
    } while (0)
    while (ok) {
        GLL_GV_PT(11);
        const int pub = (it + 1) & 1;
        const __amdgpu_buffer_rsrc_t rvp = pub ? rv1 : rv0;
        const __amdgpu_buffer_rsrc_t rpp = pub ? rpt1 : rpt0;
        if constexpr (MODE == 1) {   // w = A u, u published before the last barrier
            const __amdgpu_buffer_rsrc_t rvu = pub ? rv0 : rv1;
#pragma unroll
            for (int k = 0; k < RPG; ++k) {
                const int uu = r0 + grp + k * NG;
                if (uu < r1) {
                    const f32x4 o = spmv(k, rvu);
                    w[k] = Mat::kSeparateDiag ? dg[k] * u[k] + o : o;
                }
            }
        }
        // ---- local: partial (r,u), (w,u), (r,r); publish m = M w (pipelined form)
        {
            f32x4 pg = {0.f, 0.f, 0.f, 0.f}, pd = pg, pr = pg;
#pragma unroll
            for (int k = 0; k < RPG; ++k) {
                const int uu = r0 + grp + k * NG;
                if (uu < r1 && qown) {
                    pg += r[k] * u[k];
                    pd += w[k] * u[k];
                    pr += r[k] * r[k];
                    if constexpr (MODE == 0)
                        __builtin_amdgcn_raw_buffer_store_b128(mi[k] * w[k], rvp,
                                                               uu * rowB + 16 * li, 0, kSc1);
                }
            }
            // lanes of one quad across the wave's row groups, then the waves in order
#pragma unroll
            for (int o = LPR; o < kWave; o <<= 1) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    pg[t] += __shfl_xor(pg[t], o);
                    pd[t] += __shfl_xor(pd[t], o);
                    pr[t] += __shfl_xor(pr[t], o);
                }
            }
            if (lane < LPR && qown) {
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int c = 4 * li + t;
                    if (c < C) {
                        s_wp[wv][c] = pg[t];
                        s_wp[wv][C + c] = pd[t];
                        s_wp[wv][2 * C + c] = pr[t];
                    }
                }
            }
            __syncthreads();
            if (threadIdx.x < PW / 4) {
                f32x4 v = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int w_ = 0; w_ < NW; ++w_) v += quad_of(s_wp[w_], threadIdx.x);
                __builtin_amdgcn_raw_buffer_store_b128(v, rpp, (blockIdx.x * PW + 4 * threadIdx.x) * 4,
                                                       0, kSc1);
            }
        }
        GLL_GV_PT(12);
        ok = gv_barrier(a.sync, ++epoch, G, a.hier, &s_ok);
        GLL_GV_PT(13);
        if (a.diag_fail && it == 2) ok = false;   // injected failure (uniform over the grid)
        if (!ok) break;
        if (it == 0) GLL_TRACE_PT(9);
        // ---- the partials of every workgroup (all loads in flight; out-of-range -> 0) ...
        const int NQP = PW / 4;
        f32x4 pl[JP];
#pragma unroll
        for (int j = 0; j < JP; ++j)
            pl[j] = __builtin_amdgcn_raw_buffer_load_b128(rpp, (threadIdx.x + NT * j) * 16, 0, kSc1);
        // ---- ... while n = A m gathers the published m
        f32x4 nn[RPG];
#pragma unroll
        for (int k = 0; k < RPG; ++k) {
            const int uu = r0 + grp + k * NG;
            nn[k] = f32x4{0.f, 0.f, 0.f, 0.f};
            if (MODE == 0 && uu < r1) {
                const f32x4 o = spmv(k, rvp);
                nn[k] = Mat::kSeparateDiag ? dg[k] * (mi[k] * w[k]) + o : o;
            }
        }
        GLL_GV_PT(14);
        // slot q = threadIdx % NQP: fixed order over j, then lanes, then waves
        {
            f32x4 v = pl[0];
#pragma unroll
            for (int j = 1; j < JP; ++j) v += pl[j];
            for (int o = NQP; o < kWave; o <<= 1) {
#pragma unroll
                for (int t = 0; t < 4; ++t) v[t] += __shfl_xor(v[t], o);
            }
            if (lane < NQP) s_red[wv][lane] = v;
            __syncthreads();
        }
        GLL_GV_PT(15);
        // ---- step sizes: lane c of every wave for column c, from the waves' sums added in
        //      wave order (round 3 had one wave compute them and broadcast through LDS: two
        //      more workgroup barriers per iteration)
        float al_c = 0.f, be_c = 0.f;
        bool any;
        {
            const int c = lane;
            if (c < C) {
                const float* q0 = reinterpret_cast<const float*>(&s_red[0][0]);
                float gam = q0[c], del = q0[C + c], rho = q0[2 * C + c];
#pragma unroll
                for (int w_ = 1; w_ < NW; ++w_) {
                    const float* q = reinterpret_cast<const float*>(&s_red[w_][0]);
                    gam += q[c];
                    del += q[C + c];
                    rho += q[2 * C + c];
                }
                if (it == 0) {
                    const float tl = fmaxf(a.atol, a.rtol * sqrtf(rho));
                    tol2_c = tl * tl;
                }
                if (act_c == 1 && rho <= tol2_c) act_c = 0;   // converged
                if (act_c == 1) {
                    float den = del, be = 0.f;
                    if (it > 0) {
                        be = gam / gold_c;
                        den = del - be * gam / aold_c;
                    }
                    if (!(den > 0.f) || !(gam > 0.f)) {
                        act_c = 2;   // breakdown / NaN: stops, not converged
                    } else {
                        al_c = gam / den;
                        be_c = be;
                        gold_c = gam;
                        aold_c = al_c;
                    }
                }
            }
            any = __ballot(c < C && act_c == 1) != 0ull && it < a.max_iter;
        }
        GLL_GV_PT(16);
        if (!any) break;
        f32x4 al, be;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            al[t] = __shfl(al_c, (4 * li + t) & (kWave - 1));
            be[t] = __shfl(be_c, (4 * li + t) & (kWave - 1));
        }
        if constexpr (MODE == 0) {   // ---- local updates (Ghysels-Vanroose recurrences)
#pragma unroll
            for (int k = 0; k < RPG; ++k) {
                const int uu = r0 + grp + k * NG;
                if (uu >= r1 || !qown) continue;
                const f32x4 mk = mi[k] * w[k];
                z[k] = nn[k] + be * z[k];
                q[k] = mk + be * q[k];
                s[k] = w[k] + be * s[k];
                p[k] = u[k] + be * p[k];
                x[k] += al * p[k];
                r[k] -= al * s[k];
                u[k] -= al * q[k];
                w[k] -= al * z[k];
            }
        } else {   // ---- Chronopoulos-Gear: p, s = A p by recurrence; u = M r published
#pragma unroll
            for (int k = 0; k < RPG; ++k) {
                const int uu = r0 + grp + k * NG;
                if (uu >= r1 || !qown) continue;
                p[k] = u[k] + be * p[k];
                s[k] = w[k] + be * s[k];
                x[k] += al * p[k];
                r[k] -= al * s[k];
                u[k] = mi[k] * r[k];
                __builtin_amdgcn_raw_buffer_store_b128(u[k], rvp, uu * rowB + 16 * li, 0, kSc1);
            }
            ok = gv_barrier(a.sync, ++epoch, G, a.hier, &s_ok);
        }
        GLL_GV_PT(17);
        ++it;
    }
#undef GLL_GV_PT
#undef GLL_GV_WG
    GLL_TRACE_PT(10);
    // a failed grid barrier (a workgroup never arrived within ~1 s): one workgroup solves the
    // system alone (rescue_solve), the others write nothing
    if (!rescued<Mat, NT>(ok, a.sync + kSyncFail * kSyncLine, a.sync + kSyncRescue * kSyncLine,
                          a.sync + kSyncBegun * kSyncLine, a.sync + kSyncFinished * kSyncLine, A,
                          a, a.rescue, &s_ok)) {
#pragma unroll
        for (int k = 0; k < RPG; ++k) {
            const int uu = r0 + grp + k * NG;
            if (uu >= r1 || !qown) continue;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int c = 4 * li + t;
                if (c < C) {
                    const size_t i = size_t(uu) * C + c;
                    if (a.out64) st_out(a.out64 + i, double(x[k][t]));
                    if (a.out32) st_out(a.out32 + i, x[k][t]);
                }
            }
        }
        writer_done(a.sync + kSyncFinished * kSyncLine);
        const int nonconv = __popcll(__ballot(lane < C && act_c != 0));
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            if (a.st_iters) atomicMax(a.st_iters, it);
            if (a.st_nonconv && nonconv) atomicAdd(a.st_nonconv, nonconv);
        }
    }
    gv_exit(a.sync, G, &s_ok);
}

size_t grid_cg_workspace_floats(int m, int C) {
    const size_t Cp = size_t((C + 3) & ~3);
    const size_t classic = 64 + size_t(3) * m * Cp + size_t(3) * kGCM * 1024;
    const size_t gv = kSyncWords + size_t(2) * m * Cp + size_t(2) * kMaxG * 64;
    return (classic > gv ? classic : gv) + size_t(5) * m + 64;   // + the rescue vectors
}

// Workgroups of one kernel instance that can be resident at once on the whole device (the
// classic kernel, no dynamic LDS).
template <class Mat, int LPR, int RPG>
static int coresident_capacity() {
    static int cap = -1;
    if (cap < 0) {
        const int nb = occupancy_blocks(
            reinterpret_cast<const void*>(cg_grid_classic_kernel<Mat, LPR, RPG>), kGT, 0);
        cap = (nb > 0 ? nb : 1) * device_cus();
    }
    return cap;
}

// The rescue vectors sit past both grid kernels' regions (grid_cg_workspace_floats).
static size_t rescue_offset(int m, int C) {
    const size_t Cp = size_t((C + 3) & ~3);
    const size_t classic = 64 + size_t(3) * m * Cp + size_t(3) * kGCM * 1024;
    const size_t gv = kSyncWords + size_t(2) * m * Cp + size_t(2) * kMaxG * 64;
    return ((classic > gv ? classic : gv) + 63) & ~size_t(63);
}

// An ordinary launch sized within the co-resident capacity (one workgroup per CU at most, by
// its LDS slice).  hipLaunchCooperativeKernel cost more host time per launch for no residency
// the ordinary launch lacks, and under rocprofv3 a process that made one crashed at exit
// (DESIGN.md §3.2); the cooperative variant was removed in round 4.  A lost barrier (a
// workgroup kept off the GPU by other kernels) is rescued: one workgroup solves alone
// (rescue_solve, GLL_ST_GRID_RESCUED).
template <typename F, typename... Args>
static hipError_t launch_persistent(F fn, int G, int nt, size_t lds, hipStream_t s,
                                    const char* what, Args... args) {
    launch_k(fn, dim3(unsigned(G)), dim3(unsigned(nt)), lds, s, args...);
    return launch_status(what);
}

// ---- classic kernel: G workgroups of rows_per_wg rows
template <class Mat, int LPR, int RPG>
static hipError_t launch_grid(const Mat& A, GridCgArgs a, int G, float* ws, hipStream_t s) {
    a.rows_per_wg = (a.m + G - 1) / G;
    G = (a.m + a.rows_per_wg - 1) / a.rows_per_wg;
    if (G > 1024 || G > coresident_capacity<Mat, LPR, RPG>())   // partials hold 1024 workgroups
        return hipErrorCooperativeLaunchTooLarge;
    a.Cp = (a.C + 3) & ~3;
    a.sync = reinterpret_cast<unsigned*>(ws);          // 32-B block at the region's start
    a.Pbuf = ws + 64;                                   // 256-B aligned: 16-B buffer accesses
    a.Zbuf = a.Pbuf + size_t(2) * a.m * a.Cp;
    a.part = a.Zbuf + size_t(a.m) * a.Cp;
    a.rescue = ws + rescue_offset(a.m, a.C);
    hipError_t e = hipMemsetAsync(a.sync, 0, 32, s);   // barrier, fail, rescue, writers in/out
    if (e != hipSuccess) return e;
    return launch_persistent(cg_grid_classic_kernel<Mat, LPR, RPG>, G, kGT, 0, s,
                             "gridcg.hip:launch_grid", A, a);
}

// Lanes per row from the mean row length; rows per lane group (registers) and workgroups:
// the fewest rows per group that keep the grid within 64 workgroups (barrier cost grows with
// the arrivals), else within the co-resident capacity (at most 1024, the partials buffer).
template <class Mat>
static hipError_t dispatch_classic(const Mat& A, const GridCgArgs& a, int64_t nnz, float* ws,
                                   bool oversub, hipStream_t s) {
    const int64_t avg = a.m > 0 ? nnz / a.m : 0;
    const int LPR = avg <= 12 ? 4 : 8;
    const int64_t NG = kGT / LPR;
    int64_t cap = LPR == 4 ? std::min(coresident_capacity<Mat, 4, 1>(),
                                            coresident_capacity<Mat, 4, 8>())
                                 : std::min(coresident_capacity<Mat, 8, 1>(),
                                            coresident_capacity<Mat, 8, 8>());
    cap = std::min<int64_t>(cap, 1024);
    if (knob(GLL_KNOB_GRID_CAP) > 0) cap = std::min<int64_t>(cap, knob(GLL_KNOB_GRID_CAP));
    int rpg = 0;
    int64_t G = 0;
    for (int64_t lim : {std::min<int64_t>(64, cap), cap}) {
        for (int cand : {1, 2, 4, 8}) {
            const int64_t g = (a.m + NG * cand - 1) / (NG * cand);
            if (g <= lim) {
                rpg = cand;
                G = g;
                break;
            }
        }
        if (rpg) break;
    }
    if (!rpg) return hipErrorNotSupported;
    if (oversub) {
        rpg = 1;
        G = std::min<int64_t>(a.m, int64_t(1) << 20);
    }
    if (G < 1) G = 1;
#define GLL_GRID(L, R) \
    if (LPR == L && rpg == R) return launch_grid<Mat, L, R>(A, a, int(G), ws, s)
    GLL_GRID(4, 1); GLL_GRID(4, 2); GLL_GRID(4, 4); GLL_GRID(4, 8);
    GLL_GRID(8, 1); GLL_GRID(8, 2); GLL_GRID(8, 4); GLL_GRID(8, 8);
#undef GLL_GRID
    return hipErrorInvalidValue;
}

// ---- pipelined kernel
template <class Mat, int NT, int LPR, int RPG, int MODE>
static hipError_t launch_gv(const Mat& A, GvArgs a, int G, int64_t nnz, float* ws, bool zeroed,
                            hipStream_t s) {
    a.rows_per_wg = (a.m + G - 1) / G;
    G = (a.m + a.rows_per_wg - 1) / a.rows_per_wg;
    auto fn = cg_gv_kernel<Mat, NT, LPR, RPG, MODE>;
    allow_full_lds(reinterpret_cast<const void*>(fn));
    // the slice: the workgroup's share of the entries with a quarter of margin (rows beyond it
    // read the CSR), within what the static LDS leaves; unknown nnz (< 0): all of it
    const size_t stat = static_lds_bytes(reinterpret_cast<const void*>(fn));
    const size_t lds_max = (size_t(160) * 1024 - stat - 256) & ~size_t(15);
    size_t lds = lds_max;
    if (nnz >= 0) {
        const int64_t per = (nnz + G - 1) / G;
        lds = std::min(lds_max, size_t(per + per / 4 + 64) * 8);
    }
    const int nb = occupancy_blocks(reinterpret_cast<const void*>(fn), NT, lds);
    if (nb < 1 || G > kMaxG || G > device_cus()) return hipErrorCooperativeLaunchTooLarge;
    a.sync = reinterpret_cast<unsigned*>(ws);
    a.V = ws + kSyncWords;                       // 2560 B in: 256-B aligned
    a.part = a.V + size_t(2) * a.m * a.Cp;
    a.rescue = ws + rescue_offset(a.m, a.C);
    a.lds_cap = int(lds / 8);
    if (!zeroed) {   // a caller's workspace (gll_cg_csr); Luu solves: row_build / gv_exit
        const hipError_t e = hipMemsetAsync(a.sync, 0, kSyncWords * sizeof(unsigned), s);
        if (e != hipSuccess) return e;
    }
    if (debug_log())
        fprintf(stderr, "gll: grid CG (%s) G=%d rows/wg=%d NT=%d LPR=%d RPG=%d lds=%zu hier=%d\n",
                MODE == 0 ? "pipelined" : "Chronopoulos-Gear", G, a.rows_per_wg, NT, LPR, RPG, lds,
                a.hier);
    return launch_persistent(fn, G, NT, lds, s, "gridcg.hip:launch_gv", A, a);
}

// Workgroups: one per CU at most, about 16 rows each;
// lanes per row as wide as the rows per workgroup allow; up to 512 rows per workgroup (m <=
// 131,072 at 256 workgroups).  hipErrorNotSupported: no configuration holds it.
template <class Mat, int MODE>
static hipError_t dispatch_gv(const Mat& A, const GridCgArgs& c, int64_t nnz, float* ws,
                              hipStream_t s) {
    GvArgs a{};
    a.m = c.m;
    a.C = c.C;
    a.Cp = (c.C + 3) & ~3;
    a.NQ = (c.C + 3) >> 2;
    a.PW = 3 * c.C <= 32 ? 32 : 64;
    a.max_iter = c.max_iter;
    a.rtol = c.rtol;
    a.atol = c.atol;
    a.b = c.b;
    a.b_dtype = c.b_dtype;
    a.out64 = c.out64;
    a.out32 = c.out32;
    a.diag_fail = c.diag_fail;
    a.st_iters = c.st_iters;
    a.st_nonconv = c.st_nonconv;
    a.st_failed = c.st_failed;
    a.st_rescued = c.st_rescued;
    a.hier = 1;   // XCD-class hierarchical arrivals (a flat counter measured 116 against 74 us)
    int cap = std::min(kMaxG, device_cus());
    if (knob(GLL_KNOB_GRID_CAP) > 0) cap = std::min(cap, knob(GLL_KNOB_GRID_CAP));
    int G = int(std::min<int64_t>(cap, (int64_t(a.m) + 15) / 16));
    if (G < 1) G = 1;
    const int R = (a.m + G - 1) / G;
    // 256 threads while lanes per row can stay >= 4 with one row per lane group; 1024 threads
    // (16 waves: more gathers in flight per CU) for long row blocks
    const int nt = R <= 64 ? 256 : 1024;
    if (nt == 256) {
        if (R <= 16) return launch_gv<Mat, 256, 16, 1, MODE>(A, a, G, nnz, ws, c.sync_zeroed != 0, s);
        if (R <= 32) return launch_gv<Mat, 256, 8, 1, MODE>(A, a, G, nnz, ws, c.sync_zeroed != 0, s);
        if (R <= 64) return launch_gv<Mat, 256, 4, 1, MODE>(A, a, G, nnz, ws, c.sync_zeroed != 0, s);
        if (R <= 128) return launch_gv<Mat, 256, 4, 2, MODE>(A, a, G, nnz, ws, c.sync_zeroed != 0, s);
        if (R <= 256) return launch_gv<Mat, 256, 4, 4, MODE>(A, a, G, nnz, ws, c.sync_zeroed != 0, s);
    } else {
        if (R <= 64) return launch_gv<Mat, 1024, 16, 1, MODE>(A, a, G, nnz, ws, c.sync_zeroed != 0, s);
        if (R <= 128) return launch_gv<Mat, 1024, 8, 1, MODE>(A, a, G, nnz, ws, c.sync_zeroed != 0, s);
        if (R <= 256) return launch_gv<Mat, 1024, 4, 1, MODE>(A, a, G, nnz, ws, c.sync_zeroed != 0, s);
        if (R <= 512) return launch_gv<Mat, 1024, 4, 2, MODE>(A, a, G, nnz, ws, c.sync_zeroed != 0, s);
    }
    return hipErrorNotSupported;
}

// The pipelined kernel unless the oversubscription test asks for the classic sizing; past the
// pipelined kernel's row capacity, the classic kernel.
template <class Mat>
static hipError_t dispatch_grid(const Mat& A, const GridCgArgs& a, int64_t nnz, float* ws,
                                bool oversub, hipStream_t s) {
    if (!oversub) {
        // Luu solves (rtol 1e-6 relative): pipelined; general CSR (utils.laplace's refinement
        // sweeps on ill-conditioned systems): Chronopoulos-Gear
        hipError_t e;
        if constexpr (Mat::kSeparateDiag) e = dispatch_gv<Mat, 0>(A, a, nnz, ws, s);
        else e = dispatch_gv<Mat, 1>(A, a, nnz, ws, s);
        if (e != hipErrorNotSupported) return e;
    }
    return dispatch_classic(A, a, nnz < 0 ? int64_t(a.m) * 8 : nnz, ws, oversub, s);
}

hipError_t launch_cg_grid_luu(const Layout& L, void* wsp, const void* b, int b_dtype,
                              double* out64, float* out32, float rtol, float atol,
                              int max_iter, int32_t* st_nonconv, int32_t* st_iters,
                              int32_t* st_failed, hipStream_t s) {
    if (L.C > kGCM) return hipErrorNotSupported;
    LuuRows A{L.at<int32_t>(wsp, L.row_start), L.at<int32_t>(wsp, L.row_len),
              L.at<int32_t>(wsp, L.ucnt),      L.at<int32_t>(wsp, L.col),
              L.at<float>(wsp, L.w),           L.at<float>(wsp, L.diag), L.base};
    GridCgArgs a{};
    a.m = L.m;
    a.C = L.C;
    a.max_iter = max_iter;
    a.rtol = rtol;
    a.atol = atol;
    a.b = b;
    a.b_dtype = b_dtype;
    a.out64 = out64;
    a.out32 = out32;
    a.st_iters = st_iters;
    a.st_nonconv = st_nonconv;
    a.st_failed = st_failed;
    // the public words are one array (include/gll.h): GLL_ST_GRID_RESCUED beside SOLVE_FAILED
    a.st_rescued = st_failed ? st_failed - GLL_ST_SOLVE_FAILED + GLL_ST_GRID_RESCUED : nullptr;
    a.diag_fail = (L.flags & GLL_FLAG_DIAG_GRID_FAIL) ? 1 : 0;
    a.sync_zeroed = 1;   // row_build zeroed them before the forward; every solve leaves them so
    // U-block entries per row ~ 1.5 (K-1) m / n on kNN graphs (union rows, U share)
    const int64_t nnz_est = int64_t(double(L.m) * (L.K - 1) * 1.5 * double(L.m) / double(L.n)) + L.m;
    return dispatch_grid(A, a, nnz_est, L.at<float>(wsp, L.cgv),
                         (L.flags & GLL_FLAG_DIAG_GRID_OVERSUB) != 0, s);
}

hipError_t launch_cg_grid_csr(int m, int C, const int32_t* row_ptr, const int32_t* col,
                              const float* val, int64_t nnz, const float* b, float* x,
                              float atol, int max_iter, int32_t* iters, int32_t* nonconv,
                              int32_t* failed, float* ws, hipStream_t s) {
    if (C > kGCM) return hipErrorNotSupported;
    CsrRows A{row_ptr, col, val};
    GridCgArgs a{};
    a.m = m;
    a.C = C;
    a.max_iter = max_iter;
    a.rtol = 0.f;
    a.atol = atol;
    a.b = b;
    a.b_dtype = GLL_DT_F32;
    a.out32 = x;
    a.st_iters = iters;
    a.st_nonconv = nonconv;
    a.st_failed = failed;
    a.st_rescued = failed ? failed - GLL_ST_SOLVE_FAILED + GLL_ST_GRID_RESCUED : nullptr;
    return dispatch_grid(A, a, nnz, ws, false, s);
}

}  // namespace gll
