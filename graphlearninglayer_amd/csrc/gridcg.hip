// gridcg.hip -- Jacobi-preconditioned CG over the whole GPU, for systems too large for one
// workgroup per right-hand side (the Luu solves of big graphs -- stress, utils.laplace at
// n ~ 60k -- and gll_cg_csr).  Same algorithm as the per-column kernels of solve.hip and as
// stable_conjgrad (/root/reference/GLL.py:247-276, without its p-aliasing quirk): every
// column runs its own PCG with per-column step sizes, and a column is frozen once it meets
// its tolerance (GLL.py:258-268 masks alpha/beta the same way).
//
// One cooperative launch of persistent workgroups (G <= the co-resident capacity the runtime
// checks: the launch is refused, not queued, when the grid cannot be resident at once), grid
// barriers between phases:
//   A  q = A p  (LPR lanes per row, all C columns per gathered entry), partial (p, q)
//   B  x += a p, r -= a q, z = M r, partial (r, r), (r, z)
//   C  p = z + b p
// Dot products: each workgroup writes its partial sums, and after the barrier EVERY
// workgroup adds all partials in the same fixed order -- so every workgroup derives
// bitwise identical step sizes and convergence decisions (no broadcast, deterministic).
// Vectors are m x C row-major fp32 in the workspace (a gathered row is C contiguous floats).
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
};

// Hand-off discipline (cdna_hip_programming.md Guideline 16 R1; MI355X_MICROARCH.md
// "Valid forms", first table row): every byte another workgroup reads -- the published p / z
// rows and the partial sums -- is stored write-through (sc1) and loaded sc1 (16-B buffer
// accesses for the vectors), so the barrier needs neither an agent-scope release (L2
// write-back, ~1.7 us) nor an acquire (L1 invalidate, ~1.7 us).
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
        while (__hip_atomic_load(sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if ((++spins & 1023u) == 0) {
                if (__hip_atomic_load(sync + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    ok = 0;
                    break;
                }
                if (spins > (1u << 24)) {   // ~1 s: a workgroup never arrived
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
__global__ __launch_bounds__(kGT) void cg_grid_kernel(Mat A, GridCgArgs a) {
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
    // a failed grid barrier (a workgroup never arrived within ~1 s) leaves x partial: the
    // outputs become NaN and GLL_ST_SOLVE_FAILED is raised, so the failure surfaces in the
    // caller's loss at once and as an exception at the next status check -- never as a
    // plausible-looking U
    const float nanf_ = __builtin_nanf("");
#pragma unroll
    for (int k = 0; k < RPG; ++k) {
        const int u = r0 + grp + k * NG;
        if (u >= r1 || !qown) continue;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int c = 4 * li + t;
            if (c < C) {
                const size_t i = size_t(u) * C + c;
                const float xv = ok ? x[k][t] : nanf_;
                if (a.out64) a.out64[i] = double(xv);
                if (a.out32) a.out32[i] = xv;
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        int nonconv = 0;
        for (int c = 0; c < C; ++c) nonconv += s_active[c] != 0 ? 1 : 0;
        if (a.st_iters) atomicMax(a.st_iters, it);
        if (a.st_nonconv && (nonconv || !ok)) atomicAdd(a.st_nonconv, ok ? nonconv : C);
        if (!ok && a.st_failed) atomicOr(a.st_failed, 1);
    }
}

size_t grid_cg_workspace_floats(int m, int C) {
    const size_t Cp = size_t((C + 3) & ~3);
    return 64 + size_t(3) * m * Cp + size_t(3) * kGCM * 1024;
}

static int cu_count() {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0, v = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev);
        cus = v > 0 ? v : 1;
    }
    return cus;
}

// Workgroups of one kernel instance that can be resident at once on the whole device.
template <class Mat, int LPR, int RPG>
static int coresident_capacity() {
    static int cap = -1;
    if (cap < 0) {
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &nb, reinterpret_cast<const void*>(cg_grid_kernel<Mat, LPR, RPG>), kGT, 0) !=
            hipSuccess)
            nb = 1;
        (void)hipGetLastError();
        cap = (nb > 0 ? nb : 1) * cu_count();
    }
    return cap;
}

static bool coop_supported() {
    static int v = -1;
    if (v < 0) {
        int dev = 0, a = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&a, hipDeviceAttributeCooperativeLaunch, dev) != hipSuccess) a = 0;
        (void)hipGetLastError();
        const char* env = getenv("GLL_GRID_COOP");   // diagnostic A/B: 0 = ordinary launch
        v = (a != 0 && !(env && env[0] == '0')) ? 1 : 0;
    }
    return v == 1;
}

// G workgroups of rows_per_wg rows.  Cooperative launch: the runtime guarantees that all G are
// resident together or refuses the launch (hipErrorCooperativeLaunchTooLarge), so the grid
// barrier cannot wait on a workgroup that was never scheduled.  (Without cooperative-launch
// support: an ordinary launch sized within the occupancy capacity; the bounded barrier then
// turns a co-residency failure into NaN outputs + GLL_ST_SOLVE_FAILED.)
template <class Mat, int LPR, int RPG>
static hipError_t launch_grid(const Mat& A, GridCgArgs a, int G, float* ws, hipStream_t s) {
    a.rows_per_wg = (a.m + G - 1) / G;
    G = (a.m + a.rows_per_wg - 1) / a.rows_per_wg;
    a.Cp = (a.C + 3) & ~3;
    a.sync = reinterpret_cast<unsigned*>(ws);          // 16-B block at the region's start
    a.Pbuf = ws + 64;                                   // 256-B aligned: 16-B buffer accesses
    a.Zbuf = a.Pbuf + size_t(2) * a.m * a.Cp;
    a.part = a.Zbuf + size_t(a.m) * a.Cp;
    hipError_t e = hipMemsetAsync(a.sync, 0, 16, s);
    if (e != hipSuccess) return e;
    auto fn = cg_grid_kernel<Mat, LPR, RPG>;
    if (!coop_supported()) {
        if (G > coresident_capacity<Mat, LPR, RPG>()) return hipErrorCooperativeLaunchTooLarge;
        launch_k(fn, dim3(unsigned(G)), kGT, 0, s, A, a);
        return launch_status("gridcg.hip:launch_grid");
    }
    Mat Acopy = A;
    void* args[] = {&Acopy, &a};
    static const bool dbg_launch = getenv("GLL_DEBUG") != nullptr;
    if (dbg_launch)
        fprintf(stderr, "gll: grid CG cooperative launch G=%d rows/wg=%d LPR=%d RPG=%d cap=%d\n",
                G, a.rows_per_wg, LPR, RPG, coresident_capacity<Mat, LPR, RPG>());
    const ArmedLaunch armed = g_armed;   // bench timing: events around the launch
    g_armed = ArmedLaunch{};
    if (armed.kid >= 0) (void)hipEventRecord(armed.e0, s);
    e = hipLaunchCooperativeKernel(reinterpret_cast<const void*>(fn), dim3(unsigned(G)),
                                   dim3(kGT), args, 0, s);
    if (armed.kid >= 0) (void)hipEventRecord(armed.e1, s);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        static const bool dbg = getenv("GLL_DEBUG") != nullptr;
        if (dbg) fprintf(stderr, "gll: gridcg.hip:launch_grid (cooperative, G=%d): %s\n", G,
                         hipGetErrorString(e));
        return e;
    }
    return launch_status("gridcg.hip:launch_grid");
}

// Lanes per row from the mean row length; rows per lane group (registers) and workgroups:
// the fewest rows per group that keep the grid within 64 workgroups (barrier cost grows with
// the arrivals), else within the co-resident capacity.  Returns hipErrorNotSupported when no
// configuration holds the system (rows past capacity x 32 x 8): the caller then runs the
// per-column kernels with the Krylov vectors in the workspace, which take any size.
// `oversub` (GLL_FLAG_DIAG_GRID_OVERSUB, tests only) asks for twice the capacity.
template <class Mat>
static hipError_t dispatch_grid(const Mat& A, const GridCgArgs& a, int64_t nnz, float* ws,
                                bool oversub, hipStream_t s) {
    const int64_t avg = a.m > 0 ? nnz / a.m : 0;
    const int LPR = avg <= 12 ? 4 : 8;
    const int64_t NG = kGT / LPR;
    int64_t cap = LPR == 4 ? std::min(coresident_capacity<Mat, 4, 1>(),
                                            coresident_capacity<Mat, 4, 8>())
                                 : std::min(coresident_capacity<Mat, 8, 1>(),
                                            coresident_capacity<Mat, 8, 8>());
    const char* cap_env = getenv("GLL_GRID_CAP");   // tests: shrink the capacity (read per call)
    const int64_t cap_lim = cap_env ? std::max(1, atoi(cap_env)) : cap;
    cap = std::min(cap, cap_lim);
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
        // one row per workgroup: far past what the hardware can hold at once (at most 8
        // workgroups of kGT threads per CU), whatever the occupancy query under-reports
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
    a.diag_fail = (L.flags & GLL_FLAG_DIAG_GRID_FAIL) ? 1 : 0;
    // U-block entries per row ~ 1.5 (K-1) on kNN graphs (mean row length of the union)
    const int64_t nnz_est = int64_t(L.m) * (L.K - 1) * 3 / 2;
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
    return dispatch_grid(A, a, nnz, ws, false, s);
}

}  // namespace gll
